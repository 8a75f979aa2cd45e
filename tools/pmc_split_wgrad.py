import sqlite3,glob,collections,sys
for p in ('pmc1','pmc2'):
    db=glob.glob(f'gpurun_out/r5ah/{p}/**/*.db',recursive=True)[0]
    c=sqlite3.connect(db)
    rows=c.execute("select dispatch_id, counter_name, value, duration from counters_collection where kernel_name like '%gemm5_kernel<__hip_bfloat16, 1, 1, 6, 8>%' order by dispatch_id").fetchall()
    ids=sorted(set(r[0] for r in rows))
    cls={}
    for i,d in enumerate(ids):
        g=i//46; j=i%46
        cls[d]=('fc2' if j<23 else 'fc1', g, j%23)
    acc=collections.defaultdict(lambda: collections.defaultdict(list))
    dur=collections.defaultdict(dict)
    for d,n,v,du in rows:
        k,g,j=cls[d]
        if j<3: continue
        acc[k][n].append(v); dur[k][d]=du
    for k in ('fc1','fc2'):
        ds=list(dur[k].values())
        print(p,k,'n=%d'%len(ds),'us=%.1f'%(sum(ds)/len(ds)/1e3))
        for n,vs in sorted(acc[k].items()):
            print('   %-28s %.4g'%(n,sum(vs)/len(vs)))
