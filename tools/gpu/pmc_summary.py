"""Per-kernel means of rocprofv3 --pmc counter_collection.csv files (one row per dispatch x counter)."""
import csv
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for path in sys.argv[1:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        print("   " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main()
