"""TF tensor-bundle checkpoint compatibility (CPU).  Fixtures: the reference's own
checkpoint indexes (test/resnet50-cifar-ckpt-20190218/*.index; the .data blobs
were withheld upstream, so values are synthetic and only the layout is pinned)."""
import glob
import os

import numpy as np
import pytest
import torch

from distributed_tensorflow_resnet_amd.models.params import ParamStore
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec
from distributed_tensorflow_resnet_amd.utils import crc32c
from distributed_tensorflow_resnet_amd.utils import tensor_bundle as tb
from distributed_tensorflow_resnet_amd.utils.checkpoint import Saver, state_to_tf, tf_to_state

REF_DIR = "/root/reference/test/resnet50-cifar-ckpt-20190218"
REF_INDEXES = sorted(glob.glob(os.path.join(REF_DIR, "model.ckpt-*.index")))
needs_ref = pytest.mark.skipif(not REF_INDEXES, reason="reference checkpoint fixtures absent")


def test_crc32c_known_values():
    assert crc32c.value(b"123456789") == 0xE3069283
    assert crc32c.value(b"") == 0
    data = bytes(range(256)) * 10
    assert crc32c.extend(0, data) == crc32c._py_extend(0, data)
    for v in (0, 1, 0xDEADBEEF, 0xFFFFFFFF):
        assert crc32c.unmask(crc32c.mask(v)) == v


@needs_ref
@pytest.mark.parametrize("path", REF_INDEXES)
def test_index_rebuild_is_byte_identical(path):
    buf = open(path, "rb").read()
    header, entries = tb.read_index(path)
    assert header["num_shards"] == 1
    items = [(b"", tb.encode_header())]
    items += [(k.encode(), entries[k].encode()) for k in sorted(entries)]
    assert tb.build_table(items) == buf


@needs_ref
def test_our_layout_matches_reference_checkpoint(tmp_path):
    """Same 403 keys, dtypes, shapes, offsets and sizes as the reference's
    CIFAR ResNet-50 checkpoint; the data file is 6,083,416 bytes."""
    _, ref_entries = tb.read_index(REF_INDEXES[-1])
    spec = cifar_spec(50)
    store = ParamStore(spec)
    store.initialize(0)
    mom = torch.randn(store.n_train)
    tensors = state_to_tf(store, mom, 107738)
    prefix = str(tmp_path / "model.ckpt-107738")
    ours = tb.write_bundle(prefix, tensors)
    assert set(ours) == set(ref_entries)
    assert len(ours) == 403
    for k, e in ref_entries.items():
        o = ours[k]
        assert (o.dtype, o.shape, o.offset, o.size, o.shard_id) == \
               (e.dtype, e.shape, e.offset, e.size, e.shard_id), k
    assert os.path.getsize(tb.data_path(prefix)) == 6083416
    _, reread = tb.read_index(prefix)
    assert {k: (v.offset, v.size) for k, v in reread.items()} == \
           {k: (v.offset, v.size) for k, v in ref_entries.items()}


def test_roundtrip_and_restore(tmp_path):
    spec = cifar_spec(20)
    store = ParamStore(spec)
    store.initialize(3)
    mom = torch.randn(store.n_train)
    saver = Saver(str(tmp_path), max_to_keep=5)
    for step in (10, 20, 30, 40, 50, 60, 70):
        store.master.add_(0.01)
        prefix = saver.save(state_to_tf(store, mom, step), step)
    st = tb.read_checkpoint_state(str(tmp_path))
    assert st["model_checkpoint_path"] == prefix
    assert len(st["all_model_checkpoint_paths"]) == 5
    assert not os.path.exists(str(tmp_path / "model.ckpt-10.index"))
    assert tb.latest_checkpoint(str(tmp_path)) == prefix
    loaded = tb.read_bundle(prefix)
    s2 = ParamStore(spec)
    m2 = torch.zeros(s2.n_train)
    gs = tf_to_state(loaded, s2, m2)
    assert gs == 70
    assert torch.equal(s2.master, store.master)
    assert torch.equal(s2.stats, store.stats)
    assert torch.equal(m2, mom)
    # corrupted data is detected
    dp = tb.data_path(prefix)
    raw = bytearray(open(dp, "rb").read())
    raw[100] ^= 0xFF
    open(dp, "wb").write(bytes(raw))
    with pytest.raises(IOError):
        tb.read_bundle(prefix)


def test_reference_state_file_resolution(tmp_path):
    """The reference's `checkpoint` file holds absolute foreign paths
    (/Tensorflow/docker-multiple/...); latest_checkpoint falls back to the
    basename inside the directory."""
    spec = cifar_spec(8)
    store = ParamStore(spec)
    store.initialize(0)
    prefix = str(tmp_path / "model.ckpt-5")
    tb.write_bundle(prefix, state_to_tf(store, None, 5))
    with open(tmp_path / "checkpoint", "w") as fh:
        fh.write('model_checkpoint_path: "/Tensorflow/x/model.ckpt-5"\n')
    assert tb.latest_checkpoint(str(tmp_path)) == prefix
    assert set(tb.read_bundle(prefix)) == set(state_to_tf(store, None, 5))
