import json,sys
cur=None; rows={}; tots={}
for l in open(sys.argv[1]):
    if l.startswith('=='): cur=l[3:].strip(); continue
    if not l.startswith('{'): continue
    d=json.loads(l)
    if 'launch' in d: rows.setdefault(d['launch'],{})[cur]=d['us']
    else: tots[cur]=d['gemm_us_per_step']
cfgs=list(tots)
print('launch'.ljust(12), ' '.join(c[:12].rjust(12) for c in cfgs))
for k,v in rows.items(): print(k.ljust(12), ' '.join(f"{v.get(c,0):12.2f}" for c in cfgs))
print('TOTAL'.ljust(12), ' '.join(f"{tots[c]:12.1f}" for c in cfgs))
