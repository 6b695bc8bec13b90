"""Print the per-leg rates and stage times of one bench.py JSON line (for A/B runs)."""
import json
import sys


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    print(path, "headline", d.get("value"), d.get("unit"))
    for k, v in d.items():
        if not isinstance(v, dict) or "subframes_per_s" not in v:
            continue
        st = v.get("stage_ms_per_batch") or {}
        print(f"  {k}: {v['subframes_per_s']:.0f} sf/s, {v.get('ms_per_batch')} ms/batch, "
              + ", ".join(f"{s} {t:.3f}" for s, t in st.items()))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
