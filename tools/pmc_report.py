import csv, collections, sys, glob
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0]
        n = "bin_accum" if "accum" in n else ("bwd_bin" if "bwd_bin" in n else n[:30])
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, d in acc.items():
    print(n)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.0f}")
