"""Pretty-print tools/gemm_bench.py JSON lines: shape, hipBLASLt TF/s, TF/s per tile, worst error."""
import json
import sys

for line in sys.stdin:
    if not line.startswith("{"):
        continue
    r = json.loads(line)
    tiles = {k[4:]: v for k, v in r.items() if k.startswith("tile")}
    errs = [v for k, v in r.items() if k.startswith("err")]
    print(f"{r['shape']:16s} torch {r['torch_tflops']:7.1f} | " + " ".join(f"t{k}:{v:7.1f}" for k, v in tiles.items())
          + f" | maxerr {max(errs):.1e}")
