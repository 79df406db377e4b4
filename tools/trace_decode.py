"""Timeline of one decode from a rocprofv3 kernel trace (tools/gpu_dna_trace.sh):
decodes are delimited by the k_cont_reset launch (or, in older traces, by a
run of >= 8 memset launches).  usage: trace_decode.py <run_kernel_trace.csv> [index]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
starts = [i for i, r in enumerate(rows) if "k_cont_reset" in r["Kernel_Name"]]
if not starts:
    i = 0
    while i < len(rows):
        j = i
        while j < len(rows) and "fillBuffer" in rows[j]["Kernel_Name"]:
            j += 1
        if j - i >= 8:
            starts.append(i)
        i = max(j, i + 1)
a, b = starts[k], starts[k + 1] if k + 1 < len(starts) else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
busy, agg, last = 0, {}, t0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ldpc::dev::", "")[:44]
    c = agg.setdefault(n, [0, 0.0])
    c[0] += 1
    c[1] += (e - s) / 1000
    busy += e - s
    print(f"{(s - t0) / 1000:8.1f} {n:44s} {(e - s) / 1000:6.1f}")
    last = e
print(f"decodes {len(starts)}; span {(last - t0) / 1000:.1f} us, kernels busy {busy / 1000:.1f} us")
for n, (c, tt) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {n:44s} {c:3d} {tt:8.1f}")
