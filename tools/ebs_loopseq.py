#!/usr/bin/env python3
"""Loads / waitcnts / branches of one loop of a .s file in program order.
    python tools/ebs_loopseq.py file.s BB1_107"""
import re, sys
lines = open(sys.argv[1]).read().split('\n')
hdr = sys.argv[2]
inloop = False
for l in lines:
    m = re.match(r'^(\.LBB\d+_\d+|; %bb\.\d+):', l)
    if m:
        inloop = ('Header=' + hdr) in l or m.group(1) == '.L' + hdr
        continue
    if inloop:
        s = l.strip()
        if s.startswith(('global_load', 's_waitcnt', 's_cbranch', 's_branch')):
            print(s[:60])
