"""Per-kernel launch statistics of one rocprofv3 --kernel-trace run of bench.py, split into the
bench's two profiling windows (tools/prof_window.py): the timed region's launches and the
isolated kernel pass's.  usage: kernel_stats.py TRACE_DIR OUT_PREFIX
writes OUT_PREFIX_{timed,isolated}.txt / .csv (calls, average, min, max, total, share)."""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_window import WINDOWS, rows_of, select  # noqa: E402


def main():
    rows = rows_of(sys.argv[1], "*kernel_trace.csv")
    for which in WINDOWS:
        per = defaultdict(list)
        for r in select(rows, which):
            per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        tot = sum(sum(v) for v in per.values()) or 1
        items = sorted(per.items(), key=lambda kv: -sum(kv[1]))
        with open(f"{sys.argv[2]}_{which}.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "AverageNs", "MinNs", "MaxNs", "TotalNs", "Percentage"])
            for k, v in items:
                w.writerow([k, len(v), sum(v) / len(v), min(v), max(v), sum(v), 100.0 * sum(v) / tot])
        with open(f"{sys.argv[2]}_{which}.txt", "w") as f:
            f.write(f"rocprofv3 --kernel-trace -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline: "
                    f"the {which} window's launches (between bench.py's ProfMarks markers)\n")
            f.write(f"{'kernel':100s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}\n")
            for k, v in items:
                f.write(f"{k[:100]:100s} {len(v):6d} {sum(v) / len(v) / 1e3:9.2f} {min(v) / 1e3:9.2f} "
                        f"{max(v) / 1e3:9.2f} {100.0 * sum(v) / tot:6.2f}\n")
        print(f"== {which}: {sum(len(v) for v in per.values())} launches")
        for k, v in items[:8]:
            print(f"{k[:70]:70s} {len(v):5d} {sum(v) / len(v) / 1e3:9.2f} us")


if __name__ == "__main__":
    main()
