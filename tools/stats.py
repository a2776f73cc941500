"""Print a rocprofv3 kernel_stats.csv as a table (name, calls, average microseconds)."""
import csv
import sys

for f in sys.argv[1:]:
    print(f)
    for r in csv.DictReader(open(f)):
        print("  %-70s %5s %10.2f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
