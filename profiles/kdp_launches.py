"""Split the k_dp dispatches of a rocprofv3 kernel trace into the main
mapping launches and the mate-rescue launches (the k_dp right after a
k_rescue): rocprofv3's kernel stats average both under one name, bench.py's
roofline averages the main launches.

    python profiles/kdp_launches.py <run_kernel_trace.csv> <out.json>
"""
import csv
import json
import sys


def main(trace, out):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r['Start_Timestamp']))
    main_ms, rescue_ms = [], []
    prev = None
    for r in rows:
        name = r['Kernel_Name']
        if name.startswith('k_dp'):
            ms = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
            (rescue_ms if prev is not None and prev.startswith('k_rescue') else main_ms).append(ms)
        if not name.startswith('__amd'):
            prev = name

    def summary(v):
        return {'launches': len(v), 'avg_ms': round(sum(v) / len(v), 4) if v else None,
                'ms': [round(x, 4) for x in v]}

    res = {'source': trace, 'main': summary(main_ms), 'rescue': summary(rescue_ms),
           'all': summary(main_ms + rescue_ms)}
    with open(out, 'w') as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k]['avg_ms'] for k in ('main', 'rescue', 'all')}))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
