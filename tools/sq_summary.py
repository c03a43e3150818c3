"""SQ counter summary of the chain kernels from a rocprofv3 --pmc database:
instructions per wave and the wave-cycle split (SQ_* count quad-cycles)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else "tg_"
rows = c.execute("select kernel_name, counter_name, sum(value) from counters_collection "
                 f"where kernel_name like '%hyg::{pat}%' group by kernel_name, counter_name").fetchall()
by = {}
for k, n, v in rows:
    by.setdefault(k.split("(")[0].replace("void ", ""), {})[n] = v
for k, d in by.items():
    w = d.get("SQ_WAVES", 1) or 1
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k}: waves={w:.0f} VALU/wave={d.get('SQ_INSTS_VALU', 0) / w:.4g} SALU/wave={d.get('SQ_INSTS_SALU', 0) / w:.4g} "
          f"LDS/wave={d.get('SQ_INSTS_LDS', 0) / w:.4g} | wave cycles: waiting {d.get('SQ_WAIT_ANY', 0) / wc:.1%} "
          f"issue-stalled {d.get('SQ_WAIT_INST_ANY', 0) / wc:.1%} issuing {d.get('SQ_ACTIVE_INST_ANY', 0) / wc:.1%}")
    others = {n: v / w for n, v in d.items() if n not in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                                                          "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
    print("   per wave:", {n: round(v) for n, v in sorted(others.items())})
