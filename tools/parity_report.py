"""Summarises the measured parity errors the GPU tests log (CDX_PARITY_LOG=<file> pytest -m gpu):
per test (parameters folded) and quantity, the largest measured relative error next to its
tolerance.  The tolerances in tests/ are set ~10× the measured values from this report.

  python tools/parity_report.py gpurun_out/parity.jsonl > profiles/<tag>_parity_errors.txt
"""
import collections
import json
import sys


def main(path):
    worst = collections.defaultdict(lambda: [0.0, None, ""])
    for line in open(path):
        r = json.loads(line)
        test = r["test"].split("::")[-1]
        key = (test.split("[")[0], r["tag"])
        w = worst[key]
        if r["err"] >= w[0]:
            worst[key] = [r["err"], r["tol"], test]
    print(f"{'test':58s} {'quantity':16s} {'max rel err':>12s} {'tol':>8s}  worst case")
    for (test, tag), (err, tol, case) in sorted(worst.items()):
        print(f"{test:58s} {tag:16s} {err:12.3e} {tol:8.0e}  {case}")


if __name__ == "__main__":
    main(sys.argv[1])
