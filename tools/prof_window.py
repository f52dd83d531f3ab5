"""The bench's profiling windows in a rocprofv3 CSV (kernel_trace.csv or counter_collection.csv).

bench.py brackets its timed region and its isolated kernel pass with one marker kernel each side
(ProfMarks: torch.cuda._sleep -> `spin_kernel`, launched after a device sync and followed by
one).  Dispatch ids are assigned at enqueue, in submission order, so every launch of the timed
region has an id between the first two markers and every launch of the isolated pass one between
the last two, whatever stream it ran on.  This replaces rocprofv3 --selected-regions, which in
r05b recorded nothing with --kernel-trace and everything with --pmc."""
import csv
import glob
import os

MARKER = "spin_kernel"
WINDOWS = ("timed", "isolated")


def rows_of(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        out.extend(csv.DictReader(open(f)))
    return out


def window_ids(rows):
    """{'timed': (lo, hi), 'isolated': (lo, hi)} from the marker dispatches (exclusive bounds)."""
    marks = sorted({int(r["Dispatch_Id"]) for r in rows if MARKER in r["Kernel_Name"]})
    if len(marks) != 4:
        raise SystemExit(f"prof_window: expected 4 `{MARKER}` marker dispatches, found {len(marks)}")
    return {"timed": (marks[0], marks[1]), "isolated": (marks[2], marks[3])}


def select(rows, which):
    lo, hi = window_ids(rows)[which]
    return [r for r in rows if lo < int(r["Dispatch_Id"]) < hi]


# kernel name fragments -> the bench's short names (bench.py roofline keys)
SHORT = {"roi_sweep_kernel": "roi_align", "nchw_to_nhwc4_kernel": "nchw_to_nhwc", "nchw_to_nhwc_kernel": "nchw_to_nhwc",
         "g1dw4_kernel": "enc_g1_dwconv", "rmb_front3_kernel": "enc_rmb_front", "trans4_kernel": "enc_gemm_trans",
         "gemm4_kernel<0": "enc_gemm_dsc", "gemm4_kernel<1": "enc_gemm_trans", "enc_se_kernel": "enc_se",
         "enc_head_kernel": "enc_head", "cost_kernel": "cost", "cost3_kernel": "cost", "det_prep_kernel": "cost_prep",
         "lsap_kernel": "lsap", "step_begin_kernel": "step_begin", "step_mid_kernel": "step_mid",
         "step_end_kernel": "step_end", "step_apply_kernel": "step_apply"}


def short_name(kernel):
    return next((v for p, v in SHORT.items() if p in kernel), None)
