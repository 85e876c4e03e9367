"""Summarise rocprofv3 counter_collection.csv files: per kernel (name prefix), the median over
dispatches of each counter.  python tools/pmc_summary.py file.csv [...]"""
import collections
import csv
import statistics
import sys


def main():
    for f in sys.argv[1:]:
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:70]
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), k)
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"== {f}")
        for k, cs in vals.items():
            print("  " + k)
            for c, v in sorted(cs.items()):
                print(f"     {c:28s} median {statistics.median(v):14.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
