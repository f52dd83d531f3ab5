"""Average FETCH_SIZE / WRITE_SIZE per launch of each kernel from two
rocprofv3 --pmc passes (counter_collection.csv).  FETCH_SIZE is reported in
KiB by rocprofv3 and, on gfx950, tallies 64 B per 128-B request of wide
streaming reads (MI355X_MICROARCH.md §HBM): the corrected read bytes are
2 x FETCH_SIZE x 1024 for 16-B/lane loads; other widths are uncalibrated."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    fe, wr = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fe) | set(wr)):
        f = fe.get(k, []); w = wr.get(k, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        out[k] = dict(launches=len(f) or len(w), fetch_kib=fk, write_kib=wk,
                      read_bytes_corrected=2 * fk * 1024 if fk is not None else None,
                      write_bytes=wk * 1024 if wk is not None else None)
    short = sorted(out.items(), key=lambda kv: -((kv[1]["fetch_kib"] or 0) + (kv[1]["write_kib"] or 0)))
    for k, v in short[:20]:
        print(f"{k[:90]:90s} n={v['launches']:4d} fetch={v['fetch_kib'] or 0:12.1f} KiB write={v['write_kib'] or 0:12.1f} KiB")
    print("JSON " + json.dumps(out))


if __name__ == "__main__":
    main()
