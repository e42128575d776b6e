"""Instruction mix of the horizon loop (the backward-branch loop containing v_sin_f32)
of each rollout_kernel / chain_rollout_kernel instantiation in a device .s file.
Usage: loopstat.py file.s [-v]   (-v: the loop's opcode histogram)"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for fn in re.findall(r'^(_ZN12_GLOBAL__N_1\d+(?:chain_)?rollout_kernel\S*):', s, re.M):
    i = s.index(fn + ':')
    j = s.index('.Lfunc_end', i)
    body = s[i:j].split('\n')
    labels = {m.group(1): n for n, l in enumerate(body) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
    loops = []
    for n, l in enumerate(body):
        m = re.search(r's_cbranch_\w+\s+(\.LBB\S+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < n:
            seg = body[labels[m.group(1)]:n + 1]
            if any('v_sin_f32' in x for x in seg):
                loops.append(seg)
    if not loops:
        continue
    seg = max(loops, key=len)
    ins = [l.split()[0] for l in seg if l.strip() and not l.strip().startswith(('.', ';'))]
    c = Counter(ins)
    nsin = c['v_sin_f32_e32']
    links = 7 if 'chain' in fn and 'ILi7E' in fn else (int(re.search(r'ILi(\d)E', fn).group(1)) if 'chain' in fn else 2)
    steps = max(1, nsin // links)
    valu = sum(v for k, v in c.items() if k.startswith('v_'))
    short = re.sub(r'_ZN12_GLOBAL__N_1\d+|EEEv.*', '', fn)
    print(f"{short}: {len(ins)} instrs / {steps} steps = {len(ins)/steps:.1f} per step "
          f"(VALU {valu/steps:.1f}, s_waitcnt {c['s_waitcnt']/steps:.1f}, s_nop {c['s_nop']/steps:.1f})")
    print('   ', ', '.join(f'{k} {v/steps:.1f}' for k, v in sorted(c.items(), key=lambda x: -x[1])[:16]))
    if '-v' in sys.argv:
        print("   " + " ".join(f"{k}:{v}" for k, v in c.most_common(24)))
