"""Per-kernel SQ counter averages from two rocprofv3 --pmc passes (tools/gpu_round.sh),
with the derived rates the north star asks for:
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
              (MFMA-pipe busy cycles summed over SIMDs, MI355X_MICROARCH.md: = 32 x N_mfma for
              32x32x16 bf16; GRBM_GUI_ACTIVE sums the 8 XCDs, so / 8 = the dispatch's clocks)
  wait / issue-stall / active shares of SQ_WAVE_CYCLES (quad-cycle counters, disjoint).
usage: pmc_sq_summary.py PASS1_DIR PASS2_DIR OUT.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHORT = {"roi_sweep_kernel": "roi_align", "nchw_to_nhwc_kernel": "nchw_to_nhwc", "g1dw_kernel": "enc_g1_dwconv", "g1dw4_kernel": "enc_g1_dwconv", "rmb_front_kernel": "enc_rmb_front", "rmb_front2_kernel": "enc_rmb_front", "rmb_front3_kernel": "enc_rmb_front", "rmb_fused_kernel": "enc_rmb_fused", "trans4_kernel": "enc_gemm_trans", "gemm4w_trans_kernel": "enc_gemm_trans",
         "gemm4_kernel<0": "enc_gemm_dsc", "gemm4_kernel<1": "enc_gemm_trans", "enc_se_kernel": "enc_se",
         "enc_head_kernel": "enc_head", "cost_kernel": "cost", "cost3_kernel": "cost", "det_prep_kernel": "cost_prep", "lsap_kernel": "lsap",
         "step_begin_kernel": "step_begin", "step_mid_kernel": "step_mid", "step_end_kernel": "step_end",
         "step_apply_kernel": "step_apply"}


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
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
        json.dump({"source": "rocprofv3 --pmc (two SQ passes, kernel trace only) over bench.py --steps 5 --warmup 2; "
                             "per-launch averages; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024)",
                   "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
