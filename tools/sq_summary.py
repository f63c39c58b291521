import csv,glob,collections,sys
for d in sys.argv[1:]:
    print('==',d)
    acc=collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("p1","p2"):
        for f in glob.glob(f"{d}/{p}/**/*counter_collection.csv",recursive=True):
            for r in csv.DictReader(open(f)):
                n=r.get("Kernel_Name","")
                if "swap_loop" in n and "true, true" not in n and "<true" not in n:
                    acc[n[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n,cs in acc.items():
        print(n)
        for c,v in sorted(cs.items()):
            print(f"  {c}: {sum(v)/len(v):.4g} (n={len(v)})")
