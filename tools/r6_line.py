"""Print the headline fields of a bench.py JSON line (last line of the file)."""
import json
import sys

for path in sys.argv[1:]:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    ks = " ".join("%s %.3f" % (k, v["avg_ms"]) for k, v in (d.get("kernels") or {}).items())
    print("%s: %.3f ms/step (first %s, steady %s, kernels %s) | %s" % (
        path.split("/")[-1], d["ms_per_step"], d.get("step_ms_first"), d.get("step_ms_steady"),
        d.get("gpu_kernel_ms_per_step"), ks))
