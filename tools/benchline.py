"""Print the key figures of one bench.py JSON line: python tools/benchline.py FILE [TAG]."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tag = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
one = d.get("one_stack_in_flight") or {}
roof = d.get("roofline") or {}
print(f"{tag}: {d['value']:.1f} Mpts/s  {d['ms_per_step']:.3f} ms/step  "
      f"one-stack {one.get('ms_per_step')} ms  steady {(d.get('steady_state') or {}).get('ms_per_step')}"
      f"  K5 {roof.get('avg_ms')} ms frac {roof.get('frac')}")
print("   stage_ms", d.get("stage_ms"))
