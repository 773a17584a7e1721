"""Summarise a rocprofv3 kernel trace: mean duration per (kernel, grid)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for x in rows:
    d[(x['Kernel_Name'][:48], x['Grid_Size_X'], x['Workgroup_Size_X'], x['LDS_Block_Size'], x['VGPR_Count'])].append(
        (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print('%-48s grid=%-8s wg=%-4s lds=%-6s vgpr=%-4s n=%-4d mean=%8.2fus min=%8.2f' % (k + (len(v), sum(v) / len(v), min(v))))
