"""Per-kernel FETCH (corrected), duration and effective clock in bench.py's two profiling windows
(tools/prof_window.py: the timed region's launches and the isolated kernel pass's) from one
rocprofv3 --pmc pass that collected FETCH_SIZE, GRBM_GUI_ACTIVE and GRBM_COUNT
(counter_collection.csv carries each dispatch's start / end timestamps).  Effective clock =
GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md, DVFS give-back: reads high on
dispatches shorter than about 0.3 ms); FETCH corrected as tools/pmc_summary.py (2 x KiB x 1024).
Usage: pmc_clock.py PMC_DIR [OUT_JSON]"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_window import WINDOWS, rows_of, select, short_name  # noqa: E402


def summarise(rows):
    per = defaultdict(lambda: defaultdict(dict))  # short name -> dispatch -> counter / duration
    for r in rows:
        k = short_name(r["Kernel_Name"])
        if k is None:
            continue
        e = per[k][int(r["Dispatch_Id"])]
        e[r["Counter_Name"]] = float(r["Counter_Value"])
        e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for k, ds in per.items():
        v = list(ds.values())
        ns = sum(x["ns"] for x in v) / len(v)
        fe = [x["FETCH_SIZE"] for x in v if "FETCH_SIZE" in x]
        gr = [x["GRBM_GUI_ACTIVE"] / 8 / x["ns"] for x in v if "GRBM_GUI_ACTIVE" in x and x["ns"] > 0]
        out[k] = dict(launches=len(v), avg_us=round(ns / 1e3, 2),
                      read_bytes_corrected=round(2 * 1024 * sum(fe) / len(fe)) if fe else None,
                      clock_ghz=round(sum(gr) / len(gr), 3) if gr else None)
    return out


def main():
    rows = rows_of(sys.argv[1], "*counter_collection.csv")
    res = {"source": sys.argv[1]}
    for which in WINDOWS:
        out = summarise(select(rows, which))
        res[which] = out
        print(f"== {which}")
        for k, e in sorted(out.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["launches"]):
            print(f"{k:16s} n={e['launches']:4d} {e['avg_us']:9.2f} us  fetch "
                  f"{(e['read_bytes_corrected'] or 0) / 1e6:8.1f} MB  clock {e['clock_ghz']} GHz")
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
