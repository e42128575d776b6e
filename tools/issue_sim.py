"""In-order issue model of one wave alone on its SIMD, over a kernel's horizon loop (diagnostic, not product).

Reads the loop body that tools/loopstat.py picks, then issues it twice back to back (the second pass sees the
first pass's loop-carried results) and reports the cycles of the second pass.  An instruction issues when the
previous one has left the issue slot and its register sources are ready:
  issue cost: VALU 4 (transcendentals 8, s_nop n: 4(n+1)), SALU / waitcnt / memory 4;
  result ready after: VALU LAT (default 8), transcendental TLAT (12), SALU 4; loads are assumed in time.
Usage: issue_sim.py file.s [kernel-substring] [LAT] [TLAT] [--ubench]
--ubench: the issue costs measured by tools/ubench_issue.hip on gfx950 (profiles/r13/ubench_issue.txt, s_memtime
cycles of one wave alone): v_add 6, other VALU 7, packed 7.76, transcendental 9.8, s_nop n 6(n + 1), scalar and
memory 6; dependent-use latency LAT 9.5."""
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "chain_rollout_kernelILi7ELb1ELb0ELi4ELb0"
LAT = float(sys.argv[3]) if len(sys.argv) > 3 else 8.0
TLAT = float(sys.argv[4]) if len(sys.argv) > 4 else 12.0
fn = [f for f in re.findall(r'^(_ZN\S+):', src, re.M) if pat in f][0]
i = src.index(fn + ':')
body = src[i:src.index('.Lfunc_end', i)].split('\n')
labels = {m.group(1): n for n, l in enumerate(body) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
best = None
for n, l in enumerate(body):
    m = re.search(r's_cbranch_\w+\s+(\.LBB\S+)', l)
    if m and m.group(1) in labels and labels[m.group(1)] < n:
        seg = body[labels[m.group(1)]:n + 1]
        if any('v_sin_f32' in x for x in seg) and (best is None or len(seg) > len(best)):
            best = seg
ins = [l.strip().split(';')[0] for l in best if l.strip() and not l.strip().startswith(('.', ';'))]
TRANS = ('v_sin', 'v_cos', 'v_rsq', 'v_rcp', 'v_exp', 'v_log', 'v_sqrt')


def regs(tok):
    out = []
    for m in re.finditer(r'\b([vs])\[(\d+):(\d+)\]|\b([vs])(\d+)\b|\b(vcc|exec|scc)\b', tok):
        if m.group(1):
            out += [f"{m.group(1)}{r}" for r in range(int(m.group(2)), int(m.group(3)) + 1)]
        elif m.group(4):
            out.append(f"{m.group(4)}{m.group(5)}")
        else:
            out.append(m.group(6))
    return out


ready = {}
t = 0.0
stall = {"dep": 0.0}
op_cost = {}
start = None
for p in range(2):
    if p == 1:
        start = t
    for line in ins:
        op = line.split()[0]
        rest = line[len(op):]
        parts = [x.strip() for x in rest.split(',')]
        if op.startswith(('s_waitcnt', 's_cbranch', 's_cmp', 'global_load', 'buffer_load', 'ds_read', 'ds_write',
                          'global_store', 's_setprio')) or not parts or not parts[0]:
            dst, srcs = [], regs(rest) if op.startswith(('ds_write', 'global_store')) else []
            if op.startswith(('global_load', 'buffer_load', 'ds_read')):
                dst, srcs = regs(parts[0]), regs(','.join(parts[1:]))
        else:
            dst, srcs = regs(parts[0]), regs(','.join(parts[1:]))
        if op.startswith('v_') and ('fmac' in op or op.startswith('v_pk_fma') is False and '_dpp' in op and 'mov' not in op and False):
            srcs += dst
        if 'fmac' in op:
            srcs += dst
        if op == 's_cmp_le_i32' or op.startswith('s_cmp'):
            dst = ['scc']
        UB = '--ubench' in sys.argv
        base = 6.0 if UB else 4.0
        cost = base
        lat = base
        if op == 's_nop':
            cost = base * (int(parts[0] or 0) + 1) if parts and parts[0] else base
        elif op.startswith(TRANS):
            cost, lat = (9.8 if UB else 8.0), TLAT
        elif op.startswith('v_'):
            lat = LAT
            if UB:
                cost = 7.76 if op.startswith('v_pk_') else (6.0 if op.startswith(('v_add_f32', 'v_sub')) else 7.0)
        elif op.startswith(('global_load', 'buffer_load', 'ds_read')):
            lat = 0.0
        r = max([ready.get(s, 0.0) for s in srcs] + [t])
        if p == 1:
            stall["dep"] += r - t
            op_cost[op] = op_cost.get(op, 0.0) + cost + (r - t)
        t = r + cost
        for d in dst:
            ready[d] = t - cost + lat if lat else 0.0
cyc = t - start
print(f"{len(ins)} instrs per loop body: {cyc:.0f} cycles ({cyc / len(ins):.2f} per instr), "
      f"dependency stalls {stall['dep']:.0f} cycles (LAT {LAT}, TLAT {TLAT})")
if '-v' in sys.argv:
    for k, v in sorted(op_cost.items(), key=lambda x: -x[1])[:20]:
        print(f"   {k:24s} {v:7.0f}")
