"""One line per bench.py / bench/configs.py JSON file (gpurun summaries).

    python tools/summarize_json.py gpurun_out/r4a/*.json
"""
import json
import sys

for path in sys.argv[1:]:
    try:
        with open(path) as f:
            lines = [ln for ln in f if ln.strip().startswith("{")]
        for ln in lines:
            d = json.loads(ln)
            c = d.get("config") if isinstance(d.get("config"), dict) else d
            val = d.get("value", d.get("gpts"))
            print(path, val, c.get("transport"), c.get("cycles"), "prep", c.get("prepare_s", d.get("prepare_s")),
                  c.get("arith", d.get("arith")), "verified", d.get("verified"), "tune", c.get("autotune",
                                                                                               d.get("autotune")))
    except Exception as e:  # noqa: BLE001 - a summary never fails the run
        print(path, "unreadable:", e)
