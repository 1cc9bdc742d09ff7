"""Print a rocprofv3 kernel_stats.csv as a short table (average us, calls, name), skipping torch's
own kernels. Usage: python3 tools/kstats.py <kernel_stats.csv>..."""
import csv
import sys

for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "at::native" in n or "rocclr" in n:
            continue
        print(f"{float(r['AverageNs']) / 1000:9.1f} us  x{r['Calls']:>3}  {n[:100]}")
