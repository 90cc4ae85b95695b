"""Print a rocprofv3 kernel_stats.csv as average ms per kernel (top 12)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f"{float(r['AverageNs']) / 1e6:9.3f} ms x{r['Calls']:>3}  {r['Name'][:100]}")
