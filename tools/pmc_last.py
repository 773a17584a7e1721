"""Per kernel: the PMC counters of its LAST dispatch (the last paged batch of
tools/prof_pages.py) over the pmc5_<tag>/p_* passes; FETCH_SIZE / WRITE_SIZE
in GB (FETCH_SIZE x 2: MI355X_MICROARCH.md's gfx950 correction).
Usage: python tools/pmc_last.py <dir>"""
import csv
import glob
import sys

last = {}
for f in sorted(glob.glob(sys.argv[1] + '/p_*/**/*counter_collection.csv', recursive=True)):
    rows = list(csv.DictReader(open(f)))
    by = {}
    for x in rows:
        k = (x['Kernel_Name'].split('(')[0][:44], x['Counter_Name'])
        d = int(x['Dispatch_Id'])
        v = float(x['Counter_Value'])
        if k not in by or d > by[k][0]:
            by[k] = (d, v)
        elif d == by[k][0]:
            by[k] = (d, by[k][1] + v)
    for k, (d, v) in by.items():
        last[k] = v
names = sorted({k[0] for k in last})
ctrs = sorted({k[1] for k in last})
print('%-44s' % 'kernel' + ''.join('%16s' % c for c in ctrs))
for n in names:
    row = []
    for c in ctrs:
        v = last.get((n, c))
        if v is None:
            row.append('%16s' % '-')
        elif c == 'FETCH_SIZE':
            row.append('%13.3f GB' % (v * 2 * 1024 / 1e9))
        elif c == 'WRITE_SIZE':
            row.append('%13.3f GB' % (v * 1024 / 1e9))
        else:
            row.append('%16.0f' % v)
    print('%-44s' % n + ''.join(row))
