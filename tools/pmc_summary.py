"""Summarises rocprofv3 outputs of tools/gpu.sh into profiles/.

  python tools/pmc_summary.py TAG [E N]
Reads gpurun_out/prof_TAG (kernel-trace stats), gpurun_out/pmc_FETCH_SIZE_TAG and
gpurun_out/pmc_WRITE_SIZE_TAG (counter CSVs) and writes
  profiles/TAG_kernel_stats.csv   the rocprofv3 --stats summary (copied)
  profiles/TAG_pmc.json           per-dispatch HBM bytes per kernel, gfx950-corrected:
                                  bytes = (2·FETCH_SIZE + WRITE_SIZE)·1024 (FETCH_SIZE reads ½ of a
                                  16-B/lane coalesced stream on gfx950: MI355X_MICROARCH.md §HBM)
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(dirpath, name):
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection*.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != name:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def short(k):
    k = k.replace("void ", "").replace("(anonymous namespace)::", "")
    return k.split("(")[0]


def main():
    tag = sys.argv[1]
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    for f in glob.glob(os.path.join(out, f"prof_{tag}", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copyfile(f, os.path.join(REPO, "profiles", f"{tag}_kernel_stats.csv"))
    # steady state: the last `timed` dispatches of each kernel in the trace (the stats CSV averages
    # over the warm-up dispatches too, while the GPU clock is still ramping)
    timed = int(os.environ.get("TIMED_STEPS", "30"))
    for f in glob.glob(os.path.join(out, f"prof_{tag}", "**", "*kernel_trace.csv"), recursive=True):
        per = defaultdict(list)
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        steady = {}
        for k, v in per.items():
            v.sort()
            d = [(e - b) / 1e3 for b, e in v[-timed:]]
            steady[k] = {"dispatches_total": len(v), "last_n": len(d), "avg_us": sum(d) / len(d),
                         "min_us": min(d), "max_us": max(d)}
        json.dump({"tag": tag, "what": f"rocprofv3 kernel trace, mean over the last {timed} dispatches per kernel",
                   "kernels": steady}, open(os.path.join(REPO, "profiles", f"{tag}_kernel_steady.json"), "w"), indent=1)
    fetch = counters(os.path.join(out, f"pmc_FETCH_SIZE_{tag}"), "FETCH_SIZE")
    write = counters(os.path.join(out, f"pmc_WRITE_SIZE_{tag}"), "WRITE_SIZE")
    summary = {"tag": tag, "E": E, "n_inducing": N, "unit": "bytes per dispatch",
               "correction": "(2*FETCH_SIZE + WRITE_SIZE) * 1024", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("Cijk_") or "rocsolver" in k:
            continue  # setup-time library kernels (E11 inverse), not the hot path
        # gated launches that found nothing to do (the closure's repair pass when every check passed) move
        # a few kB: the mean is over the dispatches that moved more than 1 % of the kernel's largest one
        def live(v):
            big = [x for x in v if x > 0.01 * max(v)] if v and max(v) > 0 else v
            return big or [0]
        f = sum(live(fetch.get(k, []))) / len(live(fetch.get(k, [])))
        w = sum(live(write.get(k, []))) / len(live(write.get(k, [])))
        summary["kernels"][short(k)] = {"FETCH_SIZE_kB": f, "WRITE_SIZE_kB": w, "hbm_bytes": (2 * f + w) * 1024,
                                        "dispatches": len(fetch.get(k, [])),
                                        "dispatches_counted": len(live(fetch.get(k, [])))}
        m = re.search(r"gpis_std_kernel<\d+, (\d)", k)
        if m:  # template <KT, MODE>: 1 = whitened std pass (VAR), 2 = ∇std pass (GRADV), 3 = refine (VARL)
            key = {"1": "gpis_var_bytes_per_launch", "2": "gpis_grad_bytes_per_launch",
                   "3": "gpis_refine_bytes_per_launch"}.get(m.group(1))
            if key:
                summary[key] = (2 * f + w) * 1024
        if "gpis_screen_kernel" in k:
            summary["gpis_screen_bytes_per_launch"] = (2 * f + w) * 1024
    json.dump(summary, open(os.path.join(REPO, "profiles", f"{tag}_pmc.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))
    write_traffic(summary)


TRAFFIC_KEYS = ("gpis_screen_bytes_per_launch", "gpis_refine_bytes_per_launch", "gpis_grad_bytes_per_launch",
                "gpis_var_bytes_per_launch")


def write_traffic(summary):
    """profiles/pmc_traffic.json: the roofline kernels' HBM bytes per launch of the newest PMC run —
    the one file of profiles/ that travels to the GPU box (.gpurunignore), where bench.py puts it in
    the roofline's ``traffic`` (PMC counters cannot be read inside the timed run itself)."""
    t = {"source": f"profiles/{summary['tag']}_pmc.json", "E": summary["E"], "n_inducing": summary["n_inducing"],
         "unit": summary["unit"], "correction": summary["correction"]}
    t.update({k: summary[k] for k in TRAFFIC_KEYS if k in summary})
    json.dump(t, open(os.path.join(REPO, "profiles", "pmc_traffic.json"), "w"), indent=1)


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[1] == "--traffic-from":
    write_traffic(json.load(open(sys.argv[2])))
    sys.exit(0)


if __name__ == "__main__":
    main()
