"""Mean PMC value per (kernel, counter) over the pmc_<tag>/p* passes."""
import collections
import csv
import glob
import sys

d = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + '/p*/run_counter_collection.csv')):
    for x in csv.DictReader(open(f)):
        d[(x['Kernel_Name'][:40], x['Grid_Size'], x['Counter_Name'])].append(float(x['Counter_Value']))
for k, v in sorted(d.items()):
    print('%-40s grid=%-8s %-36s %16.1f  (n=%d)' % (k + (sum(v) / len(v), len(v))))
