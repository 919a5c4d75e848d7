#!/usr/bin/env python3
"""Average rocprofv3 counter values per kernel over the counter_collection CSVs under a directory."""
import collections
import csv
import glob
import sys


def main(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?").replace("(anonymous namespace)::", "").replace("void ", "")
            k = k.split("(")[0][-70:]
            acc[k][row.get("Counter_Name", "?")].append(float(row.get("Counter_Value", 0) or 0))
    for k, cs in sorted(acc.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
