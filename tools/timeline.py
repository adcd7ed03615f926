"""Print the GPU timeline (start/end in us from the first shown kernel) of the last N
decode steps of a rocprofv3 kernel trace, then the idle summary: per consecutive pair of
decodes, the time between one decode's last kernel and the next decode's first, and the time
in which no kernel ran on any queue over the shown window.  Developer tool.
usage: timeline.py <dir> [N] [--summary]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 3
summary_only = "--summary" in sys.argv
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
cnt = [i for i, r in enumerate(rows) if "k_decode_count" in r["Kernel_Name"]]
i0 = cnt[-n]
t0 = int(rows[i0]["Start_Timestamp"])
shown = rows[i0 - 2:]
if not summary_only:
    for r in shown:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:40]}")
# decodes: from a k_decode_prep (or count) to the k_decode_emit that follows it
dec = []
cur = None
for r in rows[cnt[-n - 1] if len(cnt) > n else cnt[0]:]:
    k = r["Kernel_Name"]
    if "k_decode_prep" in k or ("k_decode_count" in k and cur is None):
        cur = [int(r["Start_Timestamp"]), None]
    if "k_decode_emit" in k and cur is not None:
        cur[1] = int(r["End_Timestamp"])
        dec.append(cur)
        cur = None
gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(dec, dec[1:])]
# union of busy intervals over [first shown start, last end]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in shown)
busy, s0, e0 = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > e0:
        busy += e0 - s0
        s0, e0 = s, e
    else:
        e0 = max(e0, e)
busy += e0 - s0
span = max(e for _, e in iv) - iv[0][0]
print(f"decode-to-decode gaps (us): {[round(g, 1) for g in gaps]}")
print(f"window {span / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us "
      f"({(span - busy) / max(1, span) * 100:.1f} %)")
