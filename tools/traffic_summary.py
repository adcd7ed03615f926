"""Turn tools/profile_round.sh output into the files committed under profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (per-kernel durations)
  profiles/<tag>_bench.json         the bench line of the same round
  profiles/pmc_traffic.json         HBM bytes per launch of the bench's kernels, from
                                    FETCH_SIZE / WRITE_SIZE (KB), FETCH doubled per the
                                    gfx950 calibration in MI355X_MICROARCH.md (HBM section)
usage: python tools/traffic_summary.py <round dir> <tag>"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
os.makedirs(prof, exist_ok=True)
NAMES = {"k_decode_count": "decode_count", "k_decode_scan": "decode_offsets", "k_decode_emit": "decode_emit",
         "k_fast_scan": "robust_scan", "k_fast_emit": "robust_emit", "k_gather": "slice_gather",
         "k_fast_resolve": "decode_resolve", "k_expand_tiles": "plan_tiles", "k_expand_pieces": "plan_pieces"}


def short(k):
    k = k.split("(")[0].replace("void ", "")
    return k.split("::")[-1]


def per_launch(kind):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{src}/{kind}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


fetch, write = per_launch("fetch"), per_launch("write")
traffic = {}
for k, name in NAMES.items():
    if k in fetch and k in write:
        # the scan kernel is launched twice per decode (mode 1 re-runs deferred tiles only):
        # attribute the launch that does the work, i.e. the largest
        f, w = max(fetch[k]), max(write[k])
        traffic[name] = int((2 * f + w) * 1024)
        traffic[name + "_detail"] = {"fetch_kb": f, "write_kb": w, "fetch_correction": 2}
json.dump(traffic, open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
for f in glob.glob(f"{src}/trace/**/*kernel_stats.csv", recursive=True):
    shutil.copy(f, os.path.join(prof, f"{tag}_kernel_stats.csv"))
b = open(f"{src}/bench.json").read().strip().splitlines()
if b:
    open(os.path.join(prof, f"{tag}_bench.json"), "w").write(b[-1] + "\n")
print(json.dumps(traffic, indent=1))
