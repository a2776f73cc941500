import numpy as np, sys
nb=int(sys.argv[2]); raw=np.fromfile(sys.argv[1],dtype=np.uint32)
rec=raw.reshape(-1,nb,4)[-1].astype(np.int64)[:1024]
st,en,ent=rec[:,0],rec[:,1],rec[:,3]
t0=ent.min()
for nm,v in (("entry",ent),("loop start",st),("end",en)):
    u=(v-t0)/100.0; print("%-10s us: min %.1f p50 %.1f max %.1f"%(nm,u.min(),np.median(u),u.max()))
d=(st-ent)/100.0; print("prologue us: min %.1f p50 %.1f max %.1f"%(d.min(),np.median(d),d.max()))
