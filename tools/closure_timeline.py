"""Per-closure kernel timeline from a rocprofv3 kernel trace (tools/gpu.sh's prof_TAG).

  python tools/closure_timeline.py gpurun_out/prof_TAG/run_kernel_trace.csv [n_closures]

Splits the trace at each closure_queries_kernel, keeps the last n_closures full closures before the
bench's tail (default 20, skipping the last 5: the exchange and all-stage pass), and prints per
kernel position the median start / end relative to the closure's first dispatch, its duration and
stream — the gaps between the GEMM passes and the side stream's overlap read off directly.
"""
import csv
import re
import statistics as st
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:40]


def main(path, n=20):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "closure_queries_kernel" in r["Kernel_Name"]]
    seqs = [rows[a:b] for a, b in zip(idx[:-1], idx[1:])][-(n + 5):-5]
    acc = {}
    for s in seqs:
        t0 = int(s[0]["Start_Timestamp"])
        seen = {}
        for k, r in enumerate(s):
            if "closure_combine_kernel" in s[k - 1]["Kernel_Name"] and k > 0:
                break
            # a kernel is identified by (name, stream, occurrence in the closure): the side streams'
            # kernels interleave with the main stream's in a different order from closure to closure
            nm = (short(r["Kernel_Name"]), r["Stream_Id"])
            seen[nm] = seen.get(nm, 0) + 1
            acc.setdefault(nm + (seen[nm],), []).append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0))
    print(f"{len(seqs)} closures; median us relative to the closure's first dispatch (n: closures with the kernel)")
    for key in sorted(acc, key=lambda kk: st.median(x[0] for x in acc[kk])):
        v = acc[key]
        print(f"{key[0]:40s} #{key[2]} stream {key[1]}  start {st.median(x[0] for x in v) / 1e3:8.1f}"
              f"  end {st.median(x[1] for x in v) / 1e3:8.1f}  dur {st.median(x[1] - x[0] for x in v) / 1e3:7.1f}"
              f"  n {len(v)}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
