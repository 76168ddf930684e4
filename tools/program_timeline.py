import csv, sys
path, marker = sys.argv[1], sys.argv[2]
rows=list(csv.DictReader(open(path)))
ev=sorted((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),r["Kernel_Name"],r.get("Stream_Id","")) for r in rows)
spin=[i for i,e in enumerate(ev) if "spin_kernel" in e[2]]
st=[i for i,e in enumerate(ev) if marker in e[2]]
# timed steps: the 12 steps before the first probe spin that follows the timed region (the last spins are probes)
first_probe_spin = min(i for i in spin if i > st[len(st)//2]) if spin else len(ev)
sel=[s for s in st if s < first_probe_spin][-12:-1]
spans=[]
for a,b in zip(sel, sel[1:]):
    ks=ev[a:b]; t0=ks[0][0]; t1=ev[b][0]
    busy=0; cs=ce=None
    for s,e,n,_ in ks:
        if ce is None or s>ce:
            if ce is not None: busy+=ce-cs
            cs,ce=s,e
        else: ce=max(ce,e)
    busy+=ce-cs
    spans.append(((t1-t0)/1e3,busy/1e3))
print("timed steps: span", [round(a,1) for a,_ in spans], "\n busy", [round(b,1) for _,b in spans])
a,b=sel[-3],sel[-2]
ks=ev[a:b]; t0=ks[0][0]; last=t0
for s,e,n,sid in ks:
    print("%7.1f %6.1f gap %5.1f s%s %s"%((s-t0)/1e3,(e-s)/1e3,(s-last)/1e3,sid,n[:70])); last=max(last,e)
