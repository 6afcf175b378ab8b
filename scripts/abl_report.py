import csv, glob, sys
tag = sys.argv[1]
for d in sorted(glob.glob(f"gpurun_out/abl_{tag}_*/run_kernel_stats.csv")):
    name = d.split(f"abl_{tag}_")[1].split("/")[0]
    row = {r["Name"]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(d))}
    ks = {k.split("(")[0].split("::")[-1].split("<")[0]: v for k, v in row.items() if "npr::" in k}
    print(f"{name:32s} " + "  ".join(f"{k} {v:6.1f}us" for k, v in sorted(ks.items())))
