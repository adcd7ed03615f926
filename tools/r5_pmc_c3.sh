#!/bin/bash
# GPU call: HBM bytes of config 3's decode kernels (FETCH_SIZE, WRITE_SIZE: one pass each),
# 64 logs of the bench's config-3 data, sidecar on
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_c3; rm -rf $O; mkdir -p $O
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$O/p$i" -o run --output-format csv -- python3 tools/bench_config3.py --logs 64 --steps 2 > "$O/p$i.log" 2>&1 || exit $((10+i))
done
python3 - <<'P'
import csv, glob, collections, json
res = collections.defaultdict(dict)
for i, name in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
    f = glob.glob(f"gpurun_out/pmc_c3/p{i}/**/run_counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != name: continue
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        res[k][name] = sum(v) / len(v)  # KB per dispatch
out = {k: v for k, v in res.items() if any(s in k for s in ("decode_count", "decode_emit", "jser", "scatter"))}
json.dump(out, open("gpurun_out/pmc_c3/summary.json", "w"), indent=1)
for k, v in out.items():
    print(k, {n: round(x / 1024, 1) for n, x in v.items()}, "MB/dispatch")
P
