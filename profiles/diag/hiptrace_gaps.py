"""Host gaps of the last bench step in a rocprofv3 --hip-trace --kernel-trace
--memory-copy-trace run: every kernel / copy on the device timeline with the
HIP API calls the host made between them (calls under 5 us folded)."""
import csv
import sys

d = sys.argv[1]
ker = list(csv.DictReader(open(d + '/run_kernel_trace.csv')))
api = list(csv.DictReader(open(d + '/run_hip_api_trace.csv')))
cpy = list(csv.DictReader(open(d + '/run_memory_copy_trace.csv')))
def short(n):
    n = n.replace('void ', '').replace('mh::', '')
    return n.split('(')[0]


ev = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K', short(r['Kernel_Name'])) for r in ker]
ev += [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C', r.get('Direction', r.get('Kind', ''))) for r in cpy]
ev.sort()
seeds = [e for e in ev if e[3].startswith('k_seed')]
t0 = seeds[-2][0] - 200_000
t1 = max(e[1] for e in ev)
calls = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in api
               if t0 <= int(r['Start_Timestamp']) <= t1)
items = [(s, e, 'dev', k + ' ' + n) for s, e, k, n in ev if t0 <= s <= t1]
items += [(s, e, 'api', f) for s, e, f in calls if e - s >= 5000 or f in ('hipLaunchKernel', 'hipModuleLaunchKernel')]
items.sort()
base = seeds[-2][0]
for s, e, w, n in items:
    print(f"{(s - base) / 1e3:10.1f} {(e - s) / 1e3:9.1f} {w:3s} {n}")
