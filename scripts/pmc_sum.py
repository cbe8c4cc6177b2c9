#!/usr/bin/env python
"""Mean per launch of every counter, per kernel whose name starts with PREFIX:
    python scripts/pmc_sum.py COUNTER_CSV PREFIX"""
import csv
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
launches = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"^void ", "", re.sub(r"\(.*", "", r["Kernel_Name"]).strip())
    if not name.startswith(sys.argv[2]):
        continue
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    launches[name].add(r["Dispatch_Id"])
for k, cs in sorted(acc.items()):
    n = max(1, len(launches[k]))
    print(k, f"launches={n}")
    for c, v in sorted(cs.items()):
        print(f"  {c:40s} {v / n:16.1f}")
