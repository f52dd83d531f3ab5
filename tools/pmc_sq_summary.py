"""Per-kernel SQ counter averages from two rocprofv3 --pmc passes (tools/gpu_round.sh),
with the derived rates the north star asks for:
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
              (MFMA-pipe busy cycles summed over SIMDs, MI355X_MICROARCH.md: = 32 x N_mfma for
              32x32x16 bf16; GRBM_GUI_ACTIVE sums the 8 XCDs, so / 8 = the dispatch's clocks)
  wait / issue-stall / active shares of SQ_WAVE_CYCLES (quad-cycle counters, disjoint).
Only the launches of bench.py's timed region count (tools/prof_window.py).
usage: pmc_sq_summary.py PASS1_DIR PASS2_DIR OUT.json"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_window import SHORT, rows_of, select  # noqa: E402

def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for r in select(rows_of(d, "*counter_collection.csv"), "timed"):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    out = {}
    for k in set(a) | set(b):
        nm = next((v for p, v in SHORT.items() if p in k), None)
        if nm is None:
            continue
        c = {n: sum(x) / len(x) for src in (a, b) for n, x in src.get(k, {}).items()}
        g = c.get("GRBM_GUI_ACTIVE")
        e = dict(kernel=k[:120], counters={n: round(v) for n, v in sorted(c.items())})
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            e["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), 4)
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            for n, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue_stall"), ("SQ_ACTIVE_INST_ANY", "active")):
                if n in c:
                    e[lab] = round(c[n] / w, 4)
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_INSTS_LDS" in c and c["SQ_INSTS_LDS"]:
            e["lds_conflict_per_inst"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3)
        out[nm] = e
    for nm, e in sorted(out.items()):
        print(f"{nm:16s} mfma_busy={e.get('mfma_busy')} wait={e.get('wait')} stall={e.get('issue_stall')} "
              f"active={e.get('active')} lds_conf={e.get('lds_conflict_per_inst')}")
    with open(sys.argv[3], "w") as f:
        json.dump({"source": "rocprofv3 --pmc (two SQ passes, kernel trace only) over bench.py --steps 5 --warmup 2, the timed "
                             "region's launches only; "
                             "per-launch averages; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024)",
                   "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
