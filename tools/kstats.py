"""Top kernels of a rocprofv3 --stats run:  python3 tools/kstats.py DIR [N]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    print("%-72s %6s %9.1f %5.1f%%" % (r['Name'][:72], r['Calls'], float(r['AverageNs']) / 1e3,
                                       100 * float(r['TotalDurationNs']) / tot))
print("total kernel ms: %.2f" % (tot / 1e6))
