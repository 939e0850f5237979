import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_n_events' in r['Kernel_Name']]
print('k_n_events at', len(idx))
a, b = idx[-2], idx[-1]
t0 = int(rows[a]['Start_Timestamp']); t1 = int(rows[b]['Start_Timestamp'])
win = [r for r in rows if t0 - 0 <= int(r['Start_Timestamp']) < t1]
# union busy time and per-queue
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in win)
busy = 0; cur_s, cur_e = iv[0]
for s, e in iv[1:]:
    if s > cur_e: busy += cur_e - cur_s; cur_s, cur_e = s, e
    else: cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"window {(t1-t0)/1e3:.1f} us, union busy {busy/1e3:.1f} us")
for r in win:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if e - s < 20000: continue
    m = re.search(r'(k_\w+|rocprim|__amd_rocclr_\w+)', r['Kernel_Name'])
    print(f"{(s-t0)/1e3:9.1f} {(e-t0)/1e3:9.1f} {(e-s)/1e3:8.1f} q{r.get('Queue_Id','')} {m.group(1) if m else r['Kernel_Name'][:40]}")
