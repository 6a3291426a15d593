"""Count key instructions per kernel in a hipcc -S listing: python tools/isa_stats.py file.s [filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
starts = [m.start() for m in re.finditer(r'^_Z\w+:', s, re.M)]
pats = ['v_mfma', 'ds_read_b128', 'ds_read_b64_tr', 'ds_write_b128', 'global_load_dwordx4', 'global_load',
        'scratch_store', 'scratch_load', 'v_accvgpr_read', 'v_accvgpr_write', 's_barrier', 'v_exp_f32',
        's_waitcnt vmcnt', 's_waitcnt lgkmcnt']
for i, st in enumerate(starts):
    en = starts[i + 1] if i + 1 < len(starts) else len(s)
    body = s[st:en]
    name = body.split(':')[0]
    if flt not in name:
        continue
    print(name[:110])
    print("   ", {p: len(re.findall(p, body)) for p in pats})
