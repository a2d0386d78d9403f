import csv,collections,json
print(open('gpurun_out/pt.log').read().strip().splitlines()[-1])
for l in open('gpurun_out/mb_part.jsonl'): d=json.loads(l); print(d.get('filter'),d['mode'],d.get('flags'),round(d['ms_median'],3),'%.3g'%d['keys_per_s'])
rows=list(csv.DictReader(open('gpurun_out/prof_part/run_kernel_trace.csv')))
d=collections.defaultdict(list)
for r in rows:
    if 'bk_' in r['Kernel_Name'] or 'bloom_contains' in r['Kernel_Name']:
        d[r['Kernel_Name'].split('(')[0].replace('void ','')[:32]].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for n,v in d.items(): print(n, 'first10 med %.0f us'%sorted(v[:10])[5], 'last10 med %.0f'%sorted(v[-10:])[5])
