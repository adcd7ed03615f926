"""Print the GPU timeline (start/end in us from the first shown kernel) of the last N
decode steps of a rocprofv3 kernel trace.  Developer tool.  usage: timeline.py <dir> [N]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
cnt = [i for i, r in enumerate(rows) if "k_decode_count" in r["Kernel_Name"]]
i0 = cnt[-n]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0 - 2:]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:40]}")
