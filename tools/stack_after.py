#!/usr/bin/env python3
"""Run a script as __main__ and dump every thread's Python stack after N
seconds (faulthandler), then exit: where a stuck rank is waiting.

    python tools/stack_after.py SECONDS script.py [args...]
"""
import faulthandler
import runpy
import sys

secs = float(sys.argv[1])
script = sys.argv[2]
sys.argv = sys.argv[2:]
faulthandler.dump_traceback_later(secs, exit=True)
runpy.run_path(script, run_name="__main__")
