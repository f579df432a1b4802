"""Print the scorer's per-launch PMC counters from a pmc.json entry with a few
derived ratios.  usage: pmc_show.py PMC.json SCENE WID"""
import json
import sys

db = json.load(open(sys.argv[1]))
scene, wid = sys.argv[2], int(sys.argv[3])
for e in db["entries"]:
    if e["scene"] != scene or e["wid"] != wid:
        continue
    p = e["per_launch"]
    print(e["kernel"][:90])
    for k in sorted(p):
        print(f"  {k:28s} {p[k]:16.0f}")
    w = p.get("SQ_WAVES", 1)
    busy = p.get("GRBM_GUI_ACTIVE", 0)
    print(f"  VALU instr per wave {p.get('SQ_INSTS_VALU', 0) / w:.0f}, LDS instr per wave "
          f"{p.get('SQ_INSTS_LDS', 0) / w:.0f}, bank conflict cycles / LDS active "
          f"{p.get('SQ_LDS_BANK_CONFLICT', 0) / max(p.get('SQ_ACTIVE_INST_LDS', 1), 1):.2f}")
    if busy:
        print(f"  GRBM_GUI_ACTIVE {busy:.0f}: VALU busy {p.get('SQ_ACTIVE_INST_VALU', 0) * 4 / (busy * 1024):.2f} "
              f"of SIMD-cycles, MFMA busy {p.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (busy * 1024):.2f}")
