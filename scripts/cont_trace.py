"""Print the kernel sequence (name, duration) of a rocprofv3 kernel trace CSV (measurement helper)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    nm = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")[:60]
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1e6:10.3f} {(en - st) / 1e3:9.1f} us  {nm}")
