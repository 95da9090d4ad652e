"""HBM traffic per GEMM launch from the rocprofv3 PMC passes of one bench.py step
(tools/gpu.sh <tag> pmc: `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` in separate runs of
`bench.py --steps 1 --warmup 0 --grad-acc 4`).  Bytes = FETCH_SIZE x 2 (MI355X_MICROARCH.md: on
gfx950 FETCH_SIZE reports half the bytes of wide streaming reads) + WRITE_SIZE, both counted in
KiB.  Writes profiles/<name>.json, which bench.py reads for its roofline `traffic` (HBM bytes per
GEMM launch, averaged over the GEMM launches of the sampled micro-batch like `achieved`).

    python tools/traffic_summary.py gpurun_out/k_pmc1/f_counter_collection.csv \
        gpurun_out/k_pmc2/w_counter_collection.csv profiles/r01_gemm_traffic.json [WORKLOAD_JSON LIB]

WORKLOAD_JSON (bench.py's config keys: model, layers, micro_batch, seq_len, parallelism) and LIB (the
library the passes loaded: its md5 is recorded) key the file: bench.py reports the measured traffic
only on a line of the same workload run with the same library build, and `traffic: null` otherwise.
"""
import collections
import csv
import json
import sys


def per_dispatch(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1),
                                      float(r["Counter_Value"]) * 1024)
    return out


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if "<" not in name else name.split(">")[0] + ">"


GRAD_ACC = 4   # tools/gpu.sh pmc: micro-batch 3 completes a weight-gradient pair with accumulating sinks


def lib_md5(path):
    import hashlib
    with open(path, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def main(fetch, write, out, workload=None, lib=None):
    f, w = per_dispatch(fetch), per_dispatch(write)
    kinds = collections.defaultdict(list)
    gemm = []
    # the two passes are separate runs of the same deterministic program: dispatch i is the same
    # kernel in both (checked by name)
    for i, (name, wgs, fb) in f.items():
        if i not in w or w[i][0] != name:
            continue
        b = 2.0 * fb + w[i][2]
        kinds[(short(name), wgs)].append(b)
        if "gemm" in name:
            gemm.append(b)
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 1 --warmup 0 "
                     f"--grad-acc {GRAD_ACC}; bytes = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction)",
           "workload": json.loads(workload) if workload else None,
           "library_md5": lib_md5(lib) if lib else None,
           "gemm_launches": len(gemm), "gemm_avg_bytes_per_launch": sum(gemm) / max(len(gemm), 1),
           "kernels": {f"{k} [{g} WG]": {"launches": len(v), "avg_bytes": sum(v) / len(v)}
                       for (k, g), v in sorted(kinds.items(), key=lambda kv: -sum(kv[1]))[:30]}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("gemm_launches", "gemm_avg_bytes_per_launch")}))


if __name__ == "__main__":
    main(*sys.argv[1:6])
