"""Per-step GPU timeline from a rocprofv3 kernel (+ memory-copy) trace: every dispatch from one arena_upload_kernel
(the first dispatch of a query) to the next, offsets in microseconds from the step's first dispatch start."""
import csv
import sys


def main(d):
    rows = []
    for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-48:]))
    try:
        for r in csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"][12:]))
    except FileNotFoundError:
        pass
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "arena_upload" in r[2]]
    for a, b in zip(starts[-4:], starts[-3:] + [len(rows)]):
        t0 = rows[a][0]
        prev_end = rows[a - 1][1] if a else t0
        print(f"-- step (gap from previous dispatch end {(t0 - prev_end) / 1e3:.1f} us)")
        for s, e, n in rows[a:b]:
            print(f"  {(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f}  {n}")


if __name__ == "__main__":
    main(sys.argv[1])
