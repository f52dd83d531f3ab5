"""Average FETCH_SIZE / WRITE_SIZE per launch of each kernel from two
rocprofv3 --pmc passes (counter_collection.csv).  FETCH_SIZE is reported in
KiB by rocprofv3 and, on gfx950, tallies 64 B per 128-B request of wide
streaming reads (MI355X_MICROARCH.md §HBM): the corrected read bytes are
2 x FETCH_SIZE x 1024 for 16-B/lane loads; other widths are uncalibrated.  Only the launches of
bench.py's timed region count (tools/prof_window.py)."""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_window import rows_of, select  # noqa: E402


def load(d, counter):
    acc = defaultdict(list)
    if True:
        cost3 = []
        for r in select(rows_of(d, "*counter_collection.csv"), "timed"):
            if r.get("Counter_Name") != counter:
                continue
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
            if "cost3_kernel" in r["Kernel_Name"]:
                cost3.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        # the device tracker launches cost3 twice per frame, stage 1 then stage 2
        # (trk_build_cost_dev: same grid, sizes read on the device): split them by order
        cost3.sort()
        for q, (_, v) in enumerate(cost3):
            acc["cost3_kernel stage %d" % (1 + q % 2)].append(v)
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
    if len(sys.argv) > 3:  # short-name traffic table for bench.py (profiles/pmc_traffic.json)
        short_names = {"roi_sweep_kernel": "roi_align", "dwconv5_rows2_kernel": "dwconv5",
                       "dwconv5_nhwc_kernel": "dwconv5_generic", "cost_kernel": "cost", "cost3_kernel": "cost",
                       "det_prep_kernel": "cost_prep", "g1dw4_kernel": "enc_g1_dwconv",
                       "rmb_front3_kernel": "enc_rmb_front", "trans4_kernel": "enc_gemm_trans",
                       "gemm4_kernel<0": "enc_gemm_dsc", "gemm4_kernel<1": "enc_gemm_trans",
                       "enc_se_kernel": "enc_se", "enc_head_kernel": "enc_head", "det_nms_kernel": "det_nms",
                       "lsap_kernel": "lsap", "act_mean_kernel": "act_mean", "scale_rows_kernel": "scale_rows",
                       "nchw_to_nhwc_kernel": "nchw_to_nhwc", "nchw_to_nhwc4_kernel": "nchw_to_nhwc",
                       "track_update_kernel": "track_update"}
        tab = {}
        for k, v in out.items():
            if k.startswith("cost3_kernel stage"):
                if v["read_bytes_corrected"] is not None and v["write_bytes"] is not None:
                    tab["cost_stage" + k[-1]] = dict(read_bytes=round(v["read_bytes_corrected"]),
                                                    write_bytes=round(v["write_bytes"]), launches=v["launches"],
                                                    kernel=k)
                continue
            for pat, nm in short_names.items():
                if pat in k and v["read_bytes_corrected"] is not None and v["write_bytes"] is not None:
                    tab[nm] = dict(read_bytes=round(v["read_bytes_corrected"]), write_bytes=round(v["write_bytes"]),
                                   launches=v["launches"], kernel=k[:120])
        with open(sys.argv[3], "w") as f:
            json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py (separate runs), the "
                                 "timed region's launches only (tools/prof_window.py); "
                                 "read = 2 x FETCH_SIZE (gfx950 64-B tally of 128-B requests, MI355X_MICROARCH.md "
                                 "§HBM), per launch averages", "kernels": tab}, f, indent=1)


if __name__ == "__main__":
    main()
