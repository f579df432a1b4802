"""One line of an A/B log from a bench.py JSON output file.
usage: python tools/ab_line.py FILE LABEL"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sb = d.get("scaling_baseline") or {}
r = d["roofline"]
sec = d.get("secondary")
print("%s: %.3f G cand/s  step %.1f us  kernel %.1f us  pack %.1f us  with-pack step %.1f us  direct/sweep %s%s" % (
    sys.argv[2], d["value"] / 1e9, d["ms_per_step"] * 1e3, r["kernel_ms"] * 1e3, d["exchange"]["pack_us"],
    sb.get("step_ms_with_pack", float("nan")) * 1e3, (d.get("direct_path", {}).get("per_sweep"), d.get("direct_path", {}).get("numpy_order_ncc_per_sweep")),
    "" if not sec else "  | wid %d: %.3f G, kernel %.1f us, direct/sweep %s" % (
        sec["wid"], sec["value"] / 1e9, sec["kernel_ms"] * 1e3,
        (sec.get("direct_path", {}).get("per_sweep"), sec.get("direct_path", {}).get("numpy_order_ncc_per_sweep")))))
