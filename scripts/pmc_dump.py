"""Per-call averages of every counter per kernel from rocprofv3 --pmc passes (scripts/pmc_py.sh, pmc_dec.sh):
python scripts/pmc_dump.py gpurun_out/pmc_TAG [...]"""
import csv,glob,sys,collections
for out in sys.argv[1:]:
    print("==", out)
    agg=collections.defaultdict(float); n=collections.defaultdict(set); dur=collections.defaultdict(list)
    for f in glob.glob(out+"/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k=r["Kernel_Name"].split("(")[0][-60:]
            agg[(k,r["Counter_Name"])]+=float(r["Counter_Value"])
            n[(k,r["Counter_Name"])].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    for f in glob.glob(out+"/p1/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k=r["Kernel_Name"].split("(")[0][-60:]
            dur[k].append((float(r["End_Timestamp"])-float(r["Start_Timestamp"]))/1e3)
    ks=sorted({k for k,_ in agg})
    for k in ks:
        d=sorted(dur.get(k,[0])); print(k, "calls",len(d),"med us %.1f"%d[len(d)//2])
        for (kk,c),v in sorted(agg.items()):
            if kk==k: print("   %-28s %14.1f"%(c, v/len(n[(kk,c)])))
