"""Timeline of one timed step of the one-rank rehearsal from a rocprofv3 kernel trace:
python3 tools/reh_trace.py gpurun_out/<dir>/kt_kernel_trace.csv  (kernels over 0.1 ms, by queue)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:28], r['Queue_Id'],
             int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])) for r in rows)
walks = [e for e in ev if e[2].startswith('probe_walk1')]
st, en = walks[5][1], walks[7][1]
print("step ms", (en - st) / 1e6)
for s, e, n, q, g in ev:
    if s >= st and e <= en and (e - s) > 100000:
        print(f"q{q} {(s - st) / 1e6:7.2f} {(e - st) / 1e6:7.2f}  {n} ({g} WGs)")
