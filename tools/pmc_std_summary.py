"""Per-launch means of the std / screen kernels' SQ counters from tools/pmc_std.sh / pmc_screen.sh output.

  python tools/pmc_std_summary.py gpurun_out/pmc_std_<tag>   (or gpurun_out/pmc_screen_<tag>)
"""
import collections
import csv
import glob
import os
import sys


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "gpis_screen_kernel<" in k:
                agg["SCREEN"][r["Counter_Name"]].append(float(r["Counter_Value"]))
                continue
            if "gpis_std_kernel<" not in k:
                continue
            if "gpis_std_kernel<" in k and r.get("Counter_Name") is None:
                continue
            mode = k.split("gpis_std_kernel<")[1].split(",")[1].split(">")[0].strip()
            agg[{"1": "VAR", "2": "GRADV", "0": "GRAD", "3": "VARL"}[mode]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key, c in agg.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        print(key)
        for n, v in sorted(m.items()):
            print(f"  {n:30s} {v:.4g}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            # GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy is per SIMD (256 CUs × 4)
            print(f"  MFMA busy fraction            {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
            print(f"  LDS conflict / active          {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
