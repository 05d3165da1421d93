"""Print value, ms/step and per-kernel averages of gpurun_out/ab/<name>.log bench lines."""
import json
import sys

for name in sys.argv[1:]:
    for line in open(f"gpurun_out/ab/{name}.log"):
        if line.startswith("{"):
            d = json.loads(line)
            ks = {k: (v.get("ms_avg") if isinstance(v, dict) else v) for k, v in d.get("kernels", {}).items()}
            print(f"{name:8s} {d['value']:8.3f} Mtiles/s {d['ms_per_step']:7.3f} ms/step  " +
                  " ".join(f"{k}={v:.3f}" for k, v in ks.items() if isinstance(v, (int, float))))
