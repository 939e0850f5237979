"""Per-kernel timeline of the last scan step in a rocprofv3 kernel trace
(gaps between kernels show host synchronisation)."""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
first = sys.argv[2] if len(sys.argv) > 2 else 'k_n_events'
idx = [i for i, r in enumerate(rows) if first in r['Kernel_Name']]
i0 = idx[-1]
t0 = int(rows[i0]['Start_Timestamp']); prev = t0; busy = 0
for r in rows[i0:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    m = re.search(r'(k_\w+|rocprim|__amd_rocclr_\w+)', r['Kernel_Name'])
    name = m.group(1) if m else r['Kernel_Name'][:40]
    q = r.get('Queue_Id') or ''
    print(f"{(s - t0) / 1e3:9.1f} us  end {(e - t0) / 1e3:9.1f}  dur {(e - s) / 1e3:8.1f}  q{q:>3}  {name}")
    busy += e - s; prev = max(prev, e)
print(f"span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
