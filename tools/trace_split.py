"""Per-kernel split of a rocprofv3 kernel trace over a loop (tools/gpu.sh trace outputs).

  python tools/trace_split.py gpurun_out/prof_TAG/run_kernel_trace.csv ITERATIONS [MARKER]

Sums each kernel's durations over the trace window that starts at the first dispatch whose name
contains MARKER (default: the whole trace), divides by ITERATIONS, and prints a JSON object: per kernel
the µs per iteration, launches per iteration and mean µs per launch (largest first), the summed kernel
time and the wall span per iteration (their difference: gaps / host-bound time).
"""
import csv
import json
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:60]


def split(path, iters, marker=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    if marker:
        first = next(i for i, r in enumerate(rows) if marker in r["Kernel_Name"])
        rows = rows[first:]
    tot, cnt = {}, {}
    for r in rows:
        k = short(r["Kernel_Name"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[k] = tot.get(k, 0) + d
        cnt[k] = cnt.get(k, 0) + 1
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    kernels = sorted(tot, key=lambda k: -tot[k])
    return {"iterations": iters,
            "kernel_us_per_iter": sum(tot.values()) / iters / 1e3,
            "span_us_per_iter": span / iters / 1e3,
            "kernels": [{"kernel": k, "us_per_iter": tot[k] / iters / 1e3, "launches_per_iter": cnt[k] / iters,
                         "us_per_launch": tot[k] / cnt[k] / 1e3} for k in kernels]}


if __name__ == "__main__":
    print(json.dumps(split(sys.argv[1], float(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None), indent=1))
