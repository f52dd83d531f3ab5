"""Copy the judged summaries of one tools/gpu_round.sh run from gpurun_out/ into profiles/
(tracked): the kernel statistics of the timed region's and the isolated pass's launches
(tools/kernel_stats.py), the PMC traffic table (profiles/pmc_traffic.json is what bench.py's
roofline.traffic reads), the SQ pass, the FETCH + clock pass, and the bench JSON line.
usage: collect_profiles.py TAG"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
out, prof = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)


def cp(src, dst):
    s = os.path.join(out, src)
    if os.path.exists(s):
        shutil.copy(s, os.path.join(prof, dst))
        return True
    print("missing", src)
    return False


for w in ("timed", "isolated"):
    for ext in ("txt", "csv"):
        cp(f"kernel_stats_{tag}_{w}.{ext}", f"{tag}_kernel_stats_{w}.{ext}")
pm = os.path.join(out, f"pmc_traffic_{tag}.json")
if os.path.exists(pm):
    d = json.load(open(pm))
    d["profile"] = f"profiles/{tag}_pmc_traffic.json"
    json.dump(d, open(os.path.join(prof, f"{tag}_pmc_traffic.json"), "w"), indent=1)
    json.dump(d, open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
    cp(f"pmc_{tag}_summary.txt", f"{tag}_pmc_summary.txt")
cp(f"pmc_sq_{tag}.json", f"{tag}_pmc_sq.json")
cp(f"pmc_sq_{tag}.txt", f"{tag}_pmc_sq.txt")
if cp(f"pmc_clock_{tag}.json", f"{tag}_pmc_clock.json"):  # what bench.py's roofline.serialised reads
    d = json.load(open(os.path.join(out, f"pmc_clock_{tag}.json")))
    d["profile"] = f"profiles/{tag}_pmc_clock.json"
    json.dump(d, open(os.path.join(prof, "pmc_clock.json"), "w"), indent=1)
cp(f"pmc_clock_{tag}.txt", f"{tag}_pmc_clock.txt")
for name in ("bench.log", f"{tag}_bench.log"):
    p = os.path.join(out, name)
    if os.path.exists(p):
        lines = [line for line in open(p) if line.startswith("{")]
        if lines:
            open(os.path.join(prof, f"{tag}_bench.json"), "w").write(lines[-1])
for name in (f"{tag}_pytest.log", f"{tag}_smoke.log"):
    p = os.path.join(out, name)
    if os.path.exists(p):
        tail = open(p).read().splitlines()[-40:]
        open(os.path.join(prof, name.replace(".log", ".txt")), "w").write("\n".join(tail) + "\n")
print("collected", tag)
