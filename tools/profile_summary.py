"""Turn tools/profile.sh output into the files committed under profiles/.

  profiles/<tag>_bench.json                the bench line of the profile run
  profiles/<tag>_kernel_stats.csv          rocprofv3 --stats, config-2 bench (2 warm-up + 5 timed steps)
  profiles/<tag>_kernel_timed.json         per kernel: average over the LAST `steps` dispatches of the
                                           kernel trace (= the bench's timed region), to set beside the
                                           bench's own HIP-event averages
  profiles/<tag>_config3_kernel_stats.csv  rocprofv3 --stats, config 3 decode (tools/bench_config3.py)
  profiles/<tag>_inflight_kernel_stats.csv rocprofv3 --stats, the in-flight replay leg alone
  profiles/<tag>_pmc_decode.json           per config, per kernel: counters per dispatch, plus derived
                                           per-tile figures (8 KiB tiles) and HBM bytes
  profiles/pmc_traffic.json                HBM bytes per launch of the bench's kernels (bench.py reads it)

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB), FETCH doubled per the gfx950 calibration
(MI355X_MICROARCH.md, HBM section).  usage: python tools/profile_summary.py <dir> <tag>"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
TILE = 8192
STEPS = 5


def short(k):
    k = k.split("(")[0].replace("void ", "").split("::")[-1]
    return re.sub(r"<(true|false)>", lambda m: "_J" if m.group(1) == "true" else "", k)


def counters(d):
    """{kernel: {counter: [value per dispatch]}} for one pass directory."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{src}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def durations(d):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{src}/{d}/**/*kernel_trace.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            acc[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return acc


def pick(vals):
    # the decode kernels run once per step; the largest dispatch is the full batch
    return max(vals) if vals else None


def decode_table(prefix, log_bytes):
    tiles = log_bytes / TILE
    merged = collections.defaultdict(dict)
    for p in ("fetch", "write", "sq1", "sq2", "sq3"):
        for k, cs in counters(f"{prefix}_{p}").items():
            for c, v in cs.items():
                merged[k][c] = pick(v)
    dur = durations(f"{prefix}_sq1")
    out = {}
    for k, cs in sorted(merged.items()):
        if not k.startswith("k_decode") and not k.startswith("k_gather"):
            continue
        row = {"counters_per_dispatch": cs}
        d = {}
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            d["hbm_bytes"] = int((2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024)
        if k.startswith("k_decode") and "SQ_INSTS_VALU" in cs and cs.get("SQ_WAVES"):
            d["tiles"] = int(tiles)
            for c, name in (("SQ_INSTS_VALU", "valu_per_tile"), ("SQ_INSTS_SALU", "salu_per_tile"),
                            ("SQ_INSTS_LDS", "lds_per_tile"), ("SQ_INSTS_VMEM_RD", "vmem_rd_per_tile"),
                            ("SQ_INSTS_VMEM_WR", "vmem_wr_per_tile")):
                if c in cs:
                    d[name] = round(cs[c] / tiles, 1)
        if cs.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in cs:
            # lanes active per VALU cycle / 64 (1.0 = no divergence)
            d["valu_lane_util"] = round(cs["SQ_THREAD_CYCLES_VALU"] / (64 * cs["SQ_ACTIVE_INST_VALU"]), 3)
        if cs.get("SQ_INSTS_LDS"):
            d["lds_bank_conflict_per_lds_inst"] = round(cs.get("SQ_LDS_BANK_CONFLICT", 0) / cs["SQ_INSTS_LDS"], 2)
        if cs.get("SQ_WAVE_CYCLES"):
            d["wait_frac"] = round(cs.get("SQ_WAIT_ANY", 0) / cs["SQ_WAVE_CYCLES"], 3)
            d["valu_busy_frac"] = round(cs.get("SQ_ACTIVE_INST_VALU", 0) / cs["SQ_WAVE_CYCLES"], 3) \
                if "SQ_ACTIVE_INST_VALU" in cs else None
        if dur.get(k):
            d["ms_under_counters"] = round(max(dur[k]), 4)
        row["derived"] = d
        out[k] = row
    return out


os.makedirs(prof, exist_ok=True)
bench = [l for l in open(f"{src}/bench.json").read().strip().splitlines() if l.startswith("{")][-1]
open(os.path.join(prof, f"{tag}_bench.json"), "w").write(bench + "\n")
b = json.loads(bench)
for d, name in (("trace", "kernel_stats"), ("c3_trace", "config3_kernel_stats"), ("ifl_trace", "inflight_kernel_stats"),
                ("c4_trace", "config4_kernel_stats")):
    for f in glob.glob(f"{src}/{d}/**/*kernel_stats.csv", recursive=True):
        shutil.copy(f, os.path.join(prof, f"{tag}_{name}.csv"))
timed = {}
for k, v in durations("trace").items():
    last = v[-STEPS:]
    timed[k] = {"dispatches": len(v), "timed_avg_ms": round(sum(last) / len(last), 5), "all_avg_ms": round(sum(v) / len(v), 5)}
timed["note"] = ("timed_avg_ms: mean of the last %d dispatches of each kernel in the rocprofv3 kernel trace of "
                 "`bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-isolated "
                 "--no-config4 --no-config1` (the timed region); all_avg_ms includes the warm-up dispatches.  "
                 "Whether the two streams overlapped under the profiler shows in tools/timeline.py over the same "
                 "trace: compare with the bench's kernels (timed region) if they did, kernels_isolated if not" % STEPS)
json.dump(timed, open(os.path.join(prof, f"{tag}_kernel_timed.json"), "w"), indent=1)
c3_bytes = b["config3"]["log_bytes"]
pmc = {"config2": decode_table("c2", b["config"]["log_bytes_per_gpu"]),
       "config3": decode_table("c3", c3_bytes),
       "note": "max over dispatches of each counter (one full-batch decode per dispatch); tiles = log bytes / 8 KiB; "
               "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH correction)"}
json.dump(pmc, open(os.path.join(prof, f"{tag}_pmc_decode.json"), "w"), indent=1)
traffic = {}
NAMES = {"k_decode_count": "decode_count", "k_decode_emit": "decode_emit", "k_gather": "slice_gather"}
for k, name in NAMES.items():
    r = pmc["config2"].get(k, {}).get("derived", {})
    if "hbm_bytes" in r:
        traffic[name] = r["hbm_bytes"]
# provenance: the code the counters were collected on and when (bench.py reports it beside
# roofline.traffic, which it reads from this file rather than measuring in its own run)
import datetime, subprocess
try:
    head = subprocess.run(["git", "-C", os.path.dirname(prof) or ".", "rev-parse", "--short", "HEAD"],
                          capture_output=True, text=True, timeout=10).stdout.strip() or None
except Exception:
    head = None
traffic = {"kernels": traffic, "git_head": head, "tag": tag,
           "date": datetime.datetime.fromtimestamp(os.path.getmtime(f"{src}/bench.json")).strftime("%Y-%m-%d %H:%M"),
           "source": f"profiles/{tag}_pmc_decode.json (config 2, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"}
json.dump(traffic, open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
for cfg in ("config2", "config3"):
    print(cfg)
    for k, r in pmc[cfg].items():
        print(" ", k, json.dumps(r["derived"]))
print(json.dumps({k: v for k, v in timed.items() if k != "note"}, indent=0)[:1500])
