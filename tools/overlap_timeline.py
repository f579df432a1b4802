"""Timeline of a stretch of a rocprofv3 kernel trace: each kernel's start and
end (us, relative to the first kernel shown), duration, queue and stream, so
that one can read which launch a second-stream kernel queued behind.
usage: overlap_timeline.py run_kernel_trace.csv [first_kernel_index] [count] [name-filter]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
count = int(sys.argv[3]) if len(sys.argv) > 3 else 40
filt = sys.argv[4] if len(sys.argv) > 4 else ""
sel = [r for r in rows if filt in r["Kernel_Name"]][first:first + count]
t0 = int(sel[0]["Start_Timestamp"])
extra = [k for k in ("Queue_Id", "Stream_Id", "Workgroup_Size_X", "Grid_Size_X") if k in rows[0]]
print(f"{len(rows)} kernels in the trace; columns: {list(rows[0].keys())}")
for r in sel:
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:34]
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{name:34s} {(a - t0) / 1e3:9.1f} {(b - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f}  " +
          "  ".join(f"{k}={r[k]}" for k in extra))
