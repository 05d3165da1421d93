"""Study script: bench.py's per-tile line on the C5 handle (1,048,576 candidates) with a chosen library build (A/B).
Usage: c5_percall_ab.py <libANN.so> <tag> -- prints {"tag", "per_tile_calls"}."""
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import tiler_amd._lib as L
    L.LIB_PATH = os.path.abspath(sys.argv[1])
    tag = sys.argv[2]
    sys.argv = ["bench.py", "--config", "c5", "--steps", "1", "--warmup", "1", "--no-cpu", "--no-smooth", "--no-keyframes",
                "--no-dither", "--no-palettes", "--no-globaltiling", "--no-encoder"]
    import bench
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.main()
    d = json.loads(buf.getvalue().strip().splitlines()[-1])
    pt = d["secondary"]["per_tile_calls"]
    print(json.dumps({"tag": tag, "calls_per_s": pt["value"], "lone_us": pt["native"]["lone_call_us_median"],
                      "avg_batch": pt["native"]["avg_batch"], "mismatches": pt["native"]["mismatches_vs_batched"]}))


if __name__ == "__main__":
    main()
