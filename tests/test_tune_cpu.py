"""Knob hygiene: every DTR_* environment variable the code reads and every tuning
entry (native csrc/tune.cpp, engine utils/tune.py) is documented in README.md
"Knobs" with its default, the environment surface stays small, and DTR_TUNE
rejects unknown keys."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed_tensorflow_resnet_amd")

ENV_READ = re.compile(r"""(?:environ\.get\(|environ\[|getenv\(|environ\.setdefault\()\s*["'](DTR_[A-Z0-9_]+)""")
ENV_WRITE = re.compile(r"""["'](DTR_[A-Z0-9_]+)["']\s*:""")   # env dicts the launchers set
TABLE_ROW = re.compile(r"^\|\s*`([A-Za-z0-9_]+)`\s*\|\s*([^|]+?)\s*\|", re.M)


def _sources():
    files = glob.glob(os.path.join(PKG, "**", "*.py"), recursive=True)
    files += glob.glob(os.path.join(PKG, "csrc", "*.cpp")) + glob.glob(os.path.join(PKG, "csrc", "*.hip"))
    files += glob.glob(os.path.join(PKG, "csrc", "*.h"))
    files += [os.path.join(ROOT, f) for f in ("bench.py", "__graft_entry__.py")]
    files += glob.glob(os.path.join(ROOT, "*.py")) + glob.glob(os.path.join(ROOT, "launch", "**", "*.sh"),
                                                              recursive=True)
    return sorted(set(files))


def _readme_rows():
    text = open(os.path.join(ROOT, "README.md")).read()
    sec = text[text.index("## Knobs"):]
    sec = sec[:sec.index("\n## ", 4)]
    return {k: v for k, v in TABLE_ROW.findall(sec)}


def test_every_env_knob_is_documented_and_few():
    read, written = set(), set()
    for f in _sources():
        text = open(f, errors="replace").read()
        read |= set(ENV_READ.findall(text))
        written |= set(ENV_WRITE.findall(text))
    rows = _readme_rows()
    missing = sorted(k for k in read if k not in rows)
    assert not missing, f"undocumented DTR_* knobs (add them to README.md 'Knobs'): {missing}"
    assert len(read) <= 15, f"{len(read)} DTR_* environment knobs: fold tuning into DTR_TUNE"
    stale = sorted(k for k in rows if k.startswith("DTR_") and k not in read | written)
    assert not stale, f"README documents knobs no code reads: {stale}"


def _native_table():
    """(key, default) of csrc/tune.cpp's table, parsed from the source (no build needed)."""
    src = open(os.path.join(PKG, "csrc", "tune.cpp")).read()
    body = src[src.index("kTable[T_COUNT] = {"):src.index("};", src.index("kTable[T_COUNT] = {"))]
    entries = re.findall(r'\{"([a-z0-9_]+)",\s*(-?\d+),', body)
    hdr = open(os.path.join(PKG, "csrc", "tune.h")).read()
    ids = re.findall(r"^\s*(T_[A-Z0-9_]+)(?:\s*=\s*0)?,", hdr, re.M)
    assert ids and ids[-1] == "T_COUNT" or "T_COUNT" in hdr
    n_ids = len([i for i in ids if i != "T_COUNT"])
    assert len(entries) == n_ids, "tune.cpp table and tune.h TuneId enum differ in length"
    return entries


def test_every_tuning_entry_is_documented_with_its_default():
    from distributed_tensorflow_resnet_amd.utils import tune

    rows = _readme_rows()
    for key, dflt in _native_table():
        assert key in rows, f"native tuning key {key!r} missing from README.md 'Knobs'"
        assert rows[key] == dflt, f"{key}: README default {rows[key]!r} != tune.cpp {dflt!r}"
    for key, (dflt, _doc) in tune.ENGINE.items():
        assert key in rows, f"engine tuning key {key!r} missing from README.md 'Knobs'"
        assert rows[key] == str(dflt), f"{key}: README default {rows[key]!r} != {dflt!r}"
    # every tune key the native code uses is in the table (no orphan enum values)
    used = set()
    for f in (glob.glob(os.path.join(PKG, "csrc", "*.hip")) + glob.glob(os.path.join(PKG, "csrc", "*.h"))
              + glob.glob(os.path.join(PKG, "csrc", "*.cpp"))):
        used |= set(re.findall(r"\btune(?:_set)?\((T_[A-Z0-9_]+)", open(f).read()))
    hdr = open(os.path.join(PKG, "csrc", "tune.h")).read()
    declared = set(re.findall(r"^\s*(T_[A-Z0-9_]+)", hdr, re.M)) - {"T_COUNT"}
    assert used <= declared
    assert declared - used == set(), f"tuning ids nothing reads: {sorted(declared - used)}"
    # and the engine reads every engine key
    eng = open(os.path.join(PKG, "train", "engine.py")).read()
    for key in tune.ENGINE:
        assert f'tune.get("{key}")' in eng, f"engine key {key!r} is never read"


def test_dtr_tune_parsing_and_validation(monkeypatch):
    from distributed_tensorflow_resnet_amd.utils import tune

    monkeypatch.setenv("DTR_TUNE", "fork_every=2, tail_main=0.5,splitk=4")
    assert tune.get("fork_every") == 2 and tune.get("tail_main") == 0.5
    assert tune.get("stem_s2d") == 1
    tune.validate(["splitk"])
    with pytest.raises(ValueError, match="unknown DTR_TUNE"):
        tune.validate([])
    monkeypatch.setenv("DTR_TUNE", "fork_every")
    with pytest.raises(ValueError, match="not key=value"):
        tune.overrides()
    # integer keys never truncate a fractional value (strtol("12.5") == 12)
    monkeypatch.setenv("DTR_TUNE", "wgrad_slab_mb=12.5")
    with pytest.raises(ValueError, match="integer is required"):
        tune.validate(["wgrad_slab_mb"])
    monkeypatch.setenv("DTR_TUNE", "fork_every=2.5")
    with pytest.raises(ValueError, match="integer is required"):
        tune.get("fork_every")


def test_native_table_follows_the_enum_order():
    """csrc/tune.cpp's kTable is indexed by TuneId: entry i must be the key of enum entry
    i (T_FOO_BAR <-> "foo_bar"), or tune(T_X) silently reads another knob."""
    import re

    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "distributed_tensorflow_resnet_amd", "csrc")
    h = open(os.path.join(root, "tune.h")).read()
    enum = re.search(r"enum TuneId : int \{(.*?)\};", h, re.S).group(1)
    names = [n.lower()[2:] for n in re.findall(r"\b(T_[A-Z0-9_]+)", enum) if n != "T_COUNT"]
    cpp = open(os.path.join(root, "tune.cpp")).read()
    table = cpp[cpp.index("kTable[T_COUNT]"):cpp.index("std::atomic<long> g_val")]
    keys = re.findall(r'\{"([a-z0-9_]+)",', table)
    assert keys == names
