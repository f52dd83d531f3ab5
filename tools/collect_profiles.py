"""Copy the judged summaries of one tools/gpu_round.sh run from gpurun_out/ into
profiles/ (tracked): rocprofv3 kernel stats, the PMC traffic table and the
bench JSON line."""
import csv, json, os, shutil, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
out, prof = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)
src = os.path.join(out, f"prof_{tag}", "run_kernel_stats.csv")
rows = list(csv.DictReader(open(src)))
with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w") as f:
    f.write(open(src).read())
with open(os.path.join(prof, f"{tag}_kernel_stats.txt"), "w") as f:
    f.write("rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline\n")
    f.write(f"{'kernel':100s} {'calls':>6s} {'avg_us':>9s} {'pct':>6s}\n")
    for r in rows:
        f.write(f"{r['Name'][:100]:100s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} {float(r['Percentage']):6.2f}\n")
pm = os.path.join(out, f"pmc_traffic_{tag}.json")
if os.path.exists(pm):
    d = json.load(open(pm))
    d["profile"] = f"profiles/{tag}_pmc_traffic.json"
    json.dump(d, open(os.path.join(prof, f"{tag}_pmc_traffic.json"), "w"), indent=1)
    json.dump(d, open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
    shutil.copy(os.path.join(out, f"pmc_{tag}_summary.txt"), os.path.join(prof, f"{tag}_pmc_summary.txt"))
sq = os.path.join(out, f"pmc_sq_{tag}.json")
if os.path.exists(sq):
    shutil.copy(sq, os.path.join(prof, f"{tag}_pmc_sq.json"))
    shutil.copy(os.path.join(out, f"pmc_sq_{tag}.txt"), os.path.join(prof, f"{tag}_pmc_sq.txt"))
for name in ("bench.log", f"{tag}_bench.log"):
    p = os.path.join(out, name)
    if os.path.exists(p):
        lines = [l for l in open(p) if l.startswith("{")]
        if lines:
            open(os.path.join(prof, f"{tag}_bench.json"), "w").write(lines[-1])
print("collected", tag)
