#!/usr/bin/env python3
"""Does a process-wide CU mask (DTR_CU_PARTITION -> ROC_GLOBAL_CU_MASK) confine a
process's workgroups to its CUs?  Spawns one child per partition (none, 0/2, 1/2);
each child reports _C.cu_count(), the runtime's mask, and the (XCC, SE, SH, CU)
of every workgroup of a 2048-workgroup launch that spins ~50 us per wave (so the
grid spreads over every CU it may use).  The parent prints one JSON line: distinct
CUs per child and the overlap of the two halves (must be 0).

    python scripts/cu_mask_probe.py > gpurun_out/cu_mask_probe.json
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child():
    from distributed_tensorflow_resnet_amd.parallel.dist import apply_cu_partition

    mask = apply_cu_partition()
    import torch

    from distributed_tensorflow_resnet_amd import native

    nat = native(required=True)
    print(json.dumps({"mask_words_early": ["%08x" % w for w in nat.cu_mask()],
                      "cu_count": nat.cu_count()}), flush=True)
    blocks = 2048
    out = torch.zeros(2 * blocks, dtype=torch.int32, device="cuda")
    nat.cu_where(out.data_ptr(), blocks, 5000, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    v = out.view(-1, 2).cpu().tolist()
    # HW_ID: cu_id 11:8, sh_id 12, se_id 15:13; XCC_ID: low 4 bits
    cus = sorted({(x & 0xF, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 0xF) for h, x in v})
    words = nat.cu_mask()
    print(json.dumps({"partition": os.environ.get("DTR_CU_PARTITION", ""),
                      "env_mask": os.environ.get("ROC_GLOBAL_CU_MASK"),
                      "mask_words": ["%08x" % w for w in words],
                      "cu_count": nat.cu_count(), "mask_bits": sum(bin(w).count("1") for w in words),
                      "distinct_cus": len(cus), "xccs": sorted({c[0] for c in cus}),
                      "cus": cus}), flush=True)


def main():
    res = {}
    half = (1 << 128) - 1
    variants = [("", None), ("0/2", None), ("1/2", None),
                # raw mask spellings (diagnostics of the runtime's parser)
                ("raw-hi-noprefix", "%064x" % (half << 128)), ("raw-lo-noprefix", "%x" % half)]
    for part, raw in variants:
        env = dict(os.environ, DTR_CU_PARTITION=part if raw is None else "")
        env.pop("ROC_GLOBAL_CU_MASK", None)
        if raw is not None:
            env["ROC_GLOBAL_CU_MASK"] = raw
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env,
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            res[part or "none"] = {"rc": r.returncode, "err": r.stderr[-600:],
                                   "out": r.stdout[-1500:], "cus": []}
            continue
        res[part or "none"] = json.loads(r.stdout.strip().splitlines()[-1])
    a = {tuple(c) for c in res["0/2"]["cus"]}
    b = {tuple(c) for c in res["1/2"]["cus"]}
    summary = {k: {kk: vv for kk, vv in v.items() if kk != "cus"} for k, v in res.items()}
    summary["overlap_0_1"] = len(a & b)
    summary["union_0_1"] = len(a | b)
    print(json.dumps(summary), flush=True)
    return 0 if not (a & b) else 2


if __name__ == "__main__":
    sys.exit(child() if "--child" in sys.argv else main())
