"""Print a rocprofv3 kernel_stats.csv as a table (name, calls, avg/min/max us, total ms, %).
usage: python tools/prof_stats.py <run_kernel_stats.csv>"""
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:64]:64s} {int(x['Calls']):6d} avg {float(x['AverageNs'])/1e3:8.1f}us "
          f"min {float(x['MinNs'])/1e3:7.1f} max {float(x['MaxNs'])/1e3:7.1f} "
          f"tot {float(x['TotalDurationNs'])/1e6:8.2f}ms {float(x['Percentage']):6.2f}%")
