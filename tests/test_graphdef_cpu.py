"""Golden oracle from the reference's own frozen graph (CPU).

Fixture: `test/resnet50-cifar-ckpt-20190218/resnet50_cifar_frozen_model_eval.pb`
(written by the reference's resnet_cifar_frozen_model.py:111-122: the trained
CIFAR-10 ResNet-50 v2 with its 758,618 weights and 98 BN moving statistics
as Const nodes).  It is decoded data-only (utils/graphdef.py) and executed by
an independent op-by-op interpreter of TF semantics (utils/tf_interp.py), which
then pins our network builder, our CPU model and our GraphDef exporter."""
import os

import numpy as np
import pytest
import torch

from distributed_tensorflow_resnet_amd.models.params import ParamStore
from distributed_tensorflow_resnet_amd.models.resnet_torch import TorchResNet
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec, imagenet_spec
from distributed_tensorflow_resnet_amd.ops.reference import BN_EPS
from distributed_tensorflow_resnet_amd.utils import frozen
from distributed_tensorflow_resnet_amd.utils import graphdef as gd
from distributed_tensorflow_resnet_amd.utils.checkpoint import tf_to_state
from distributed_tensorflow_resnet_amd.utils.tf_interp import Interpreter

REF_DIR = "/root/reference/test/resnet50-cifar-ckpt-20190218"
REF_EVAL_META = os.path.join(REF_DIR, "resnet50_cifar_eval_graph.meta")
REF_PB = os.path.join(REF_DIR, "resnet50_cifar_frozen_model_eval.pb")
if not os.path.exists(REF_PB):   # copy kept with the tests (tests/fixtures/README.md)
    REF_PB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures",
                          "resnet50_cifar_frozen_model_eval.pb")
REF_META = os.path.join(REF_DIR, "model.ckpt-107738.meta")
needs_pb = pytest.mark.skipif(not os.path.exists(REF_PB), reason="reference frozen graph absent")


@pytest.fixture(scope="module")
def ref_graph():
    return gd.read_graph(REF_PB)


@pytest.fixture(scope="module")
def ref_tensors():
    return frozen.read_frozen(REF_PB)[1]


def _cpu_model(spec, tensors):
    store = ParamStore(spec)
    tf_to_state(tensors, store, None, strict=True)
    return TorchResNet(spec, store)


@needs_pb
def test_reference_graph_census_and_bn_epsilon(ref_graph):
    assert len(ref_graph.nodes) == 704
    assert ref_graph.op_census() == {
        "Add": 24, "ArgMax": 2, "AvgPool": 1, "BiasAdd": 1, "Cast": 1, "Const": 258,
        "Conv2D": 52, "Equal": 1, "FusedBatchNorm": 49, "Identity": 256, "MatMul": 1,
        "Mean": 1, "Pad": 4, "Placeholder": 2, "Relu": 49, "Reshape": 1, "Softmax": 1}
    eps = {n.attr["epsilon"] for n in ref_graph.nodes if n.op == "FusedBatchNorm"}
    assert eps == {float(np.float32(1.001e-5))}
    assert abs(BN_EPS - 1.001e-5) < 1e-12     # what our kernels and CPU path use


@pytest.mark.skipif(not os.path.exists(REF_META), reason="reference .meta absent")
def test_reference_training_graph_uses_same_epsilon():
    g = gd.read_meta_graph(REF_META)
    assert len(g.nodes) == 6331
    bns = [n for n in g.nodes if n.op in ("FusedBatchNorm", "FusedBatchNormGrad")]
    assert len(bns) == 98
    assert {n.attr["epsilon"] for n in bns} == {float(np.float32(1.001e-5))}
    assert {n.attr["is_training"] for n in bns} == {True}


@needs_pb
def test_spec_inferred_from_reference_graph(ref_graph, ref_tensors):
    spec = frozen.spec_from_graph(ref_graph)
    assert (spec.dataset, spec.resnet_size, spec.num_classes) == ("cifar10", 50, 10)
    n = sum(int(np.prod(p.shape)) for p in spec.trainables)
    assert n == 758618
    assert set(ref_tensors) == {p.name for p in spec.params}


@needs_pb
def test_export_reproduces_reference_graph_node_for_node(ref_graph, ref_tensors):
    ours = frozen.export_graphdef(cifar_spec(50), ref_tensors)
    assert len(ours.nodes) == len(ref_graph.nodes)
    for a, b in zip(ref_graph.nodes, ours.nodes):
        assert (a.name, a.op, a.inputs) == (b.name, b.op, b.inputs)
        assert set(a.attr) == set(b.attr), a.name
        for k, va in a.attr.items():
            vb = b.attr[k]
            if isinstance(va, np.ndarray):
                assert va.dtype == vb.dtype and va.shape == vb.shape, (a.name, k)
                assert np.array_equal(va, vb), (a.name, k)
            else:
                assert va == vb, (a.name, k, va, vb)
    # and the wire format round-trips
    back = gd.decode_graph(gd.encode_graph(ours))
    assert [(n.name, n.op, n.inputs) for n in back.nodes] == \
        [(n.name, n.op, n.inputs) for n in ours.nodes]


@needs_pb
def test_cpu_model_matches_reference_graph(ref_graph, ref_tensors):
    """Our builder + fp32 CPU model with the trained weights vs TF's graph (fp64)."""
    torch.manual_seed(0)
    x = torch.randn(8, 32, 32, 3)
    labels = torch.randint(0, 10, (8,))
    y = torch.nn.functional.one_hot(labels, 10).float()
    interp = Interpreter(ref_graph)
    probs, logits, pred, prec = interp.run(["Softmax", "final_dense", "predictions", "precision"],
                                           {"X": x, "Y": y})
    model = _cpu_model(cifar_spec(50), ref_tensors)
    with torch.no_grad():
        ours = model(x, False).double()
    rel = ((ours - logits).norm() / logits.norm()).item()
    assert rel < 1e-5, rel
    assert torch.equal(ours.argmax(1), pred)
    assert abs(float(prec) - float((pred == labels).double().mean())) < 1e-12
    assert torch.allclose(torch.softmax(ours, 1), probs, atol=1e-6)
    # trained weights: confident, non-degenerate predictions
    assert probs.max(1).values.mean() > 0.3


@needs_pb
def test_public_generator_api_matches_reference_graph(ref_graph, ref_tensors):
    """The resnet_model_official-compatible API (cifar10_resnet_v2_generator, TF
    variable names, HWIO kernels) loaded with the reference's trained weights ==
    the reference's own frozen graph run by the interpreter, in eval mode."""
    from distributed_tensorflow_resnet_amd.models import resnet_model_official as rmo

    torch.manual_seed(0)
    x = torch.randn(8, 32, 32, 3)
    model = rmo.cifar10_resnet_v2_generator(50, 10)
    with torch.no_grad():
        model(x, False)                       # creates the variables (TF creation order)
        vars_ = model.variables()
        assert set(vars_) == set(ref_tensors)
        for name, v in vars_.items():
            v.copy_(torch.from_numpy(np.asarray(ref_tensors[name], dtype=np.float32)))
        ours = model(x, False).double()
    logits = Interpreter(ref_graph).run("final_dense", {"X": x})
    rel = ((ours - logits).norm() / logits.norm()).item()
    assert rel < 1e-5, rel
    assert rmo._BATCH_NORM_EPSILON == BN_EPS


def test_imagenet_export_matches_cpu_model():
    """Stem pad 3/3 + VALID, 3x3/2 SAME max-pool, bottleneck blocks: the exported
    GraphDef run by the interpreter == our CPU model."""
    spec = imagenet_spec(0, num_classes=10, image_hw=64, block="bottleneck", layers=[1, 1, 1, 1])
    store = ParamStore(spec)
    store.initialize(3)
    g = torch.Generator().manual_seed(1)
    for s in store.stat_slots:   # non-trivial moving statistics
        v = store.view(s.name)
        v.copy_(0.1 * torch.randn(v.shape, generator=g) if s.name.endswith("mean")
                else torch.rand(v.shape, generator=g) + 0.5)
    tensors = {s.name: store.view(s.name).detach().numpy().copy()
               for s in store.train_slots + store.stat_slots}
    graph = gd.decode_graph(gd.encode_graph(frozen.export_graphdef(spec, tensors)))
    census = graph.op_census()
    assert census["MaxPool"] == 1 and census["Pad"] == 7 and census["Conv2D"] == 17
    x = torch.randn(2, 64, 64, 3, generator=g)
    logits = Interpreter(graph).run("final_dense", {"X": x})
    with torch.no_grad():
        ours = TorchResNet(spec, store)(x, False).double()
    assert logits.abs().max() > 1e-3
    assert ((ours - logits).norm() / logits.norm()).item() < 1e-5


@needs_pb
def test_freeze_writes_graphdef_and_predict_reads_reference(tmp_path, ref_tensors):
    from distributed_tensorflow_resnet_amd.models.params import ParamStore as PS
    from distributed_tensorflow_resnet_amd.utils import tensor_bundle as tb

    # checkpoint of the trained weights -> freeze -> .pb -> read back
    spec = cifar_spec(50)
    store = PS(spec)
    tf_to_state(ref_tensors, store, None, strict=True)
    tensors = dict(ref_tensors)
    tensors["global_step"] = np.array(107738, dtype=np.int64)
    prefix = str(tmp_path / "model.ckpt-107738")
    tb.write_bundle(prefix, tensors)
    out = str(tmp_path / "frozen.pb")
    meta = frozen.freeze(prefix, out, "cifar10", 50)
    assert meta["nodes"] == 704 and meta["global_step"] == 107738
    meta_path = meta["meta_graph"]
    assert os.path.basename(meta_path) == "resnet50_cifar_eval_graph.meta"
    mg = gd.read_meta_graph(meta_path)
    pbg = gd.read_graph(out)
    def _init(name):   # the variables' initializer subgraphs and Assigns (meta graph only)
        return "/Initializer" in name or name.endswith("/Assign") or name == "global_step"

    assert [n.name for n in mg.nodes if not _init(n.name)] == [n.name for n in pbg.nodes]
    pb_ops = pbg.by_name()
    params = set(ref_tensors)
    for n in mg.nodes:
        if n.name in params:
            assert n.op == "VariableV2" and pb_ops[n.name].op == "Const"
            assert list(n.attr["shape"].dims) == list(np.asarray(ref_tensors[n.name]).shape)
        elif not _init(n.name):
            assert n.op == pb_ops[n.name].op and n.inputs == pb_ops[n.name].inputs, n.name
    info = gd.read_meta_info(meta_path)
    assert info["tensorflow_version"] == "1.12.0"
    assert len(info["collections"]["trainable_variables"]) == 152
    assert len(info["collections"]["variables"]) == 251
    if os.path.exists(os.path.join(REF_DIR, "resnet50_cifar_eval_graph.meta")):
        # the reference's own eval meta graph: same variables, same creation order
        ref_info = gd.read_meta_info(os.path.join(REF_DIR, "resnet50_cifar_eval_graph.meta"))
        assert info["collections"]["trainable_variables"] == ref_info["collections"]["trainable_variables"]
        assert info["collections"]["variables"] == ref_info["collections"]["variables"]
        ref_mg = gd.read_meta_graph(os.path.join(REF_DIR, "resnet50_cifar_eval_graph.meta"))
        ref_vars = {n.name: n for n in ref_mg.nodes if n.op == "VariableV2"}
        for n in mg.nodes:
            if n.op == "VariableV2":
                assert n.attr["shape"].dims == ref_vars[n.name].attr["shape"].dims, n.name
                assert n.attr["dtype"] == ref_vars[n.name].attr["dtype"], n.name
        # every variable carries its initializer + Assign like TF's own export,
        # and the VariableDefs name them (import_meta_graph resolves initializer_name)
        ref_ops = {n.name: n.op for n in ref_mg.nodes}
        our_ops = {n.name: n.op for n in mg.nodes}
        census = lambda ops, pat: sorted(o for k, o in ops.items() if pat in k)  # noqa: E731
        assert census(our_ops, "/Initializer") == census(ref_ops, "/Initializer")
        assert census(our_ops, "/Assign") == census(ref_ops, "/Assign")
        ours_v, ref_v = gd.read_variable_defs(meta_path), gd.read_variable_defs(REF_EVAL_META)
        for key in ("variables", "trainable_variables"):
            assert ours_v[key] == ref_v[key], key
    # freezing again into the same directory keeps the existing eval meta graph
    before = open(meta_path, "rb").read()
    open(meta_path, "ab").write(b"x")
    frozen.freeze(prefix, out, "cifar10", 50)
    assert open(meta_path, "rb").read() == before + b"x"
    meta2, t2 = frozen.read_frozen(out)
    assert meta2["resnet_size"] == 50
    for k, v in ref_tensors.items():
        assert np.array_equal(v, t2[k]), k
    # the reference's own .pb through both inference paths
    x = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8)
    labels = torch.randint(0, 10, (4,))
    p_interp, prec_i = frozen.FrozenModel(REF_PB, "interp", 4).predict(x, labels)
    p_cpu, prec_c = frozen.FrozenModel(REF_PB, "cpu", 4).predict(x, labels)
    assert torch.allclose(p_interp, p_cpu, atol=1e-5)
    assert prec_i == prec_c
