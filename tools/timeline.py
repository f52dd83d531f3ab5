"""Per-step GPU timeline from a rocprofv3 kernel trace (run_kernel_trace.csv):
splits the trace at each rmb_front3_kernel launch (one per frame) and prints, for
the steps named, every kernel's stream, start offset and duration, plus the
busy fraction of the step (union of kernel intervals).
usage: python tools/timeline.py TRACE.csv [first_step] [n_steps]"""
import csv
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:48]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k0 = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nk = int(sys.argv[3]) if len(sys.argv) > 3 else 2
marks = [i for i, r in enumerate(rows) if "rmb_front3_kernel" in r["Kernel_Name"]]
print(f"{len(rows)} kernels, {len(marks)} front launches")
for s in range(k0, min(k0 + nk, len(marks) - 1)):
    a, b = marks[s], marks[s + 1]
    t0 = int(rows[a]["Start_Timestamp"]); t1 = int(rows[b]["Start_Timestamp"])
    iv = []
    print(f"--- step {s}: {(t1 - t0) / 1e3:.1f} us")
    for r in rows[a:b]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv.append((st, en))
        print(f"  q{r['Queue_Id']:>2} s{r['Stream_Id']:>2} +{(st - t0) / 1e3:8.1f} {(en - st) / 1e3:8.1f}  {short(r['Kernel_Name'])}")
    busy, cur_s, cur_e = 0, None, None
    for st, en in sorted(iv):
        if cur_e is None or st > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
    busy += cur_e - cur_s
    print(f"  busy {busy / 1e3:.1f} us of {(t1 - t0) / 1e3:.1f} ({busy / (t1 - t0):.2%})")
