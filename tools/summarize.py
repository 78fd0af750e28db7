"""Print one line per bench log: file, Mrays/s, ms/step, kernel ms, roofline frac."""
import glob
import json
import sys

for f in sorted(sys.argv[1:] or glob.glob("gpurun_out/bench_*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        r = d["roofline"]
        print(f"{f:45s} {d['value']:9.2f} Mrays/s  {d['ms_per_step']:7.3f} ms/step  "
              f"kernel {r['kernel_ms']:7.3f} ms  frac {r['frac']:.3f}")
    except Exception as e:  # noqa: BLE001
        print(f, "unparsable:", e)
