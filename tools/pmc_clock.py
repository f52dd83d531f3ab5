"""Per-kernel FETCH (corrected), duration and effective clock from one rocprofv3 --pmc pass
that collected FETCH_SIZE and GRBM_GUI_ACTIVE (counter_collection.csv, which carries each
dispatch's start / end timestamps).  Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration
(MI355X_MICROARCH.md, DVFS give-back); FETCH corrected as tools/pmc_summary.py (2 x KiB x 1024).
Usage: pmc_clock.py PMC_DIR [OUT_JSON]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter / duration
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
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
    for k, e in sorted(out.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["launches"])[:16]:
        print(f"{k[:60]:60s} n={e['launches']:4d} {e['avg_us']:9.2f} us  fetch {(e['read_bytes_corrected'] or 0) / 1e6:8.1f} MB"
              f"  clock {e['clock_ghz']} GHz")
    if len(sys.argv) > 2:
        json.dump({"source": d, "kernels": out}, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
