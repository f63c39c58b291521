#!/usr/bin/env python3
"""Lab (not shipped): one gKL2 run through the library's CLI entry
(ek_cli_main, context torn down, normal process exit) so that a profiler
attached to this process can write its output (the gKL2 executable ends
with _exit).  usage: python tools/cli_run.py HGR [args...]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(REPO, "eig-kl-algorithm_amd", "build", "libeigkl_hip.so"))
argv = [b"gKL2"] + [a.encode() for a in sys.argv[1:]]
arr = (ctypes.c_char_p * (len(argv) + 1))(*argv, None)
sys.exit(lib.ek_cli_main(b"gKL2", len(argv), arr))
