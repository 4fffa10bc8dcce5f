"""Print the last step's kernel timeline from a rocprofv3 kernel-trace CSV."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
seq = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:40]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
last = seq[-n:]
t0 = last[0][0]
for a, b, k in last:
    print("%8.1f %8.1f  %s" % ((a - t0) / 1e3, (b - a) / 1e3, k))
