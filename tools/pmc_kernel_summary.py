"""Per-dispatch means of every PMC counter for the kernels whose name contains SUBSTR, from a directory of
rocprofv3 --pmc passes (…/p*/run_counter_collection.csv), plus the derived wave-state fractions.

  python tools/pmc_kernel_summary.py gpurun_out/pmc_sdf_TAG sdf_culled
"""
import collections
import csv
import glob
import os
import sys


def main(d, sub):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
                agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in agg.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        print(k, f"({max(len(v) for v in c.values())} dispatches)")
        for n, v in sorted(m.items()):
            print(f"  {n:28s} {v:.4g}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if n in m:
                    print(f"  {n + ' / WAVE_CYCLES':42s} {m[n] / wc:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
