"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg ms, %)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    name = r["Name"].replace("(anonymous namespace)::", "")
    print(f"{name[:48]:48s} {r['Calls']:>4s} {float(r['AverageNs']) / 1e6:9.3f} ms {float(r['Percentage']):6.2f}%")
