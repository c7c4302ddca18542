#!/usr/bin/env python3
"""Where the SGPR-spill lane moves sit: for one kernel of snake_kernels.hip's
gfx950 assembly, every loop (a backward branch to an earlier label) with its
instruction count, v_writelane / v_readlane / scratch counts and the source
lines it spans (from -gline-tables-only .loc directives). VERDICT r2 item 2:
count the lane moves inside the draw-round and trace loops before changing them.

    python scripts/loop_spills.py [kernel-substring] [extra hipcc flags...]
    python scripts/loop_spills.py --sites k1 k2 ...   (one summary line per kernel)

--sites: every spill move (v_writelane into a spill VGPR, v_readlane from one)
with the source line it belongs to (the last non-zero .loc) and the innermost
loop around it (with that loop's source-line span): the moves on the per-job
path versus those inside the draw-round / trace / encode loops (VERDICT r4
item 6).
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.environ.get("SRC", os.path.join(ROOT, "marl-snake_amd", "csrc", "snake_kernels.hip"))
FLAGS = ['-O3', '-std=c++17', '-ffp-contract=off', '--offload-arch=gfx950', '-mllvm',
         '-amdgpu-atomic-optimizer-strategy=None', '--cuda-device-only', '-gline-tables-only']


def kernel_body(text, sub):
    for m in re.finditer(r'^(_Z\w+):[^\n]*$(.*?)^\.Lfunc_end', text, re.S | re.M):
        if sub in m.group(1):
            return m.group(1), m.group(2).splitlines()
    sys.exit('kernel not found: ' + sub)


def compile_asm(extra):
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, 'k.s')
        r = subprocess.run(['/opt/rocm/bin/hipcc'] + FLAGS + ['-S', SRC, '-o', asm] + extra,
                           capture_output=True, text=True)
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        return open(asm).read()


def sites(text, sub):
    """Spill moves of one kernel by source line and innermost loop."""
    name, lines = kernel_body(text, sub)
    ins, labels, cur = [], {}, 0
    for ln in lines:
        s = ln.strip()
        m = re.match(r'\.loc\s+\d+\s+(\d+)', s)
        if m:
            cur = int(m.group(1)) or cur   # (line 0: compiler-made code, keep the last line)
            continue
        m = re.match(r'^(\.LBB\w+):', s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if ln.startswith('\t') and s and not s.startswith(('.', ';')):
            ins.append((s, cur))
    spill_v = {m.group(1) for s, _ in ins for m in [re.match(r'v_writelane_b32\s+(v\d+)', s)] if m}
    loops = sorted({(labels[m.group(1)], j) for j, (s, _) in enumerate(ins)
                    for m in [re.match(r's_(?:cbranch_\w+|branch)\s+(\.LBB\w+)', s)]
                    if m and m.group(1) in labels and labels[m.group(1)] <= j})
    by = {}
    for j, (s, line) in enumerate(ins):
        st = re.match(r'v_writelane_b32\s+(v\d+)', s)
        ld = re.match(r'v_readlane_b32\s+\w+,\s*(v\d+)', s)
        if not (st or (ld and ld.group(1) in spill_v)):
            continue
        inner = min((l for l in loops if l[0] <= j <= l[1]), key=lambda l: l[1] - l[0], default=None)
        if inner:
            src = [c for _, c in ins[inner[0]:inner[1] + 1] if c]
            key = f'loop {min(src)}-{max(src)} ({inner[1] - inner[0] + 1} instructions)'
        else:
            key = 'straight-line'
        d = by.setdefault(key, {'stores': 0, 'reloads': 0, 'lines': set()})
        d['stores' if st else 'reloads'] += 1
        d['lines'].add(line)
    return {'kernel': name, 'instructions': len(ins), 'spill_vgprs': sorted(spill_v),
            'sites': {k: {'stores': v['stores'], 'reloads': v['reloads'], 'src_lines': sorted(v['lines'])}
                      for k, v in sorted(by.items())}}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == '--sites':
        text = compile_asm([])
        for sub in sys.argv[2:]:
            print(json.dumps(sites(text, sub)))
        return
    sub = sys.argv[1] if len(sys.argv) > 1 else 'k_autoresetILi4ELb0ELb0E'
    text = compile_asm(sys.argv[2:])
    name, lines = kernel_body(text, sub)
    files = {m.group(1): m.group(2) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', text, re.M)}
    # instruction stream with the current source line
    ins, labels, cur = [], {}, None
    for ln in lines:
        s = ln.strip()
        m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
        if m:
            f = files.get(m.group(1), '?')
            cur = (os.path.basename(f), int(m.group(2)))
            continue
        m = re.match(r'^(\.LBB\w+):', s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if ln.startswith('\t') and s and not s.startswith(('.', ';')):
            ins.append((s, cur))
    # spill VGPRs: the destinations of v_writelane (the code itself writes no
    # lanes); a v_readlane from one of them is a spill reload, the others are
    # the code's own broadcasts (readlane / twist neighbours)
    spill_v = {m.group(1) for s, _ in ins for m in [re.match(r'v_writelane_b32\s+(v\d+)', s)] if m}

    def reload(s):
        m = re.match(r'v_readlane_b32\s+\w+,\s*(v\d+)', s)
        return bool(m) and m.group(1) in spill_v
    loops = []
    for j, (s, _) in enumerate(ins):
        m = re.match(r's_(?:cbranch_\w+|branch)\s+(\.LBB\w+)', s)
        if m and m.group(1) in labels and labels[m.group(1)] <= j:
            loops.append((labels[m.group(1)], j))
    out = []
    for a, b in sorted(set(loops)):
        body = ins[a:b + 1]
        src = sorted({c[1] for _, c in body if c and c[0] == 'snake_kernels.hip'})
        out.append({
            'first': a, 'last': b, 'instructions': len(body),
            'v_writelane': sum(s.startswith('v_writelane') for s, _ in body),
            'v_readlane': sum(s.startswith('v_readlane') for s, _ in body),
            'spill_reloads': sum(reload(s) for s, _ in body),
            'scratch_ops': sum(s.startswith(('scratch_', 'buffer_store', 'buffer_load')) for s, _ in body),
            'src_lines': [src[0], src[-1]] if src else None,
        })
    print(json.dumps({'kernel': name, 'instructions': len(ins),
                      'v_writelane': sum(s.startswith('v_writelane') for s, _ in ins),
                      'v_readlane': sum(s.startswith('v_readlane') for s, _ in ins),
                      'spill_reloads': sum(reload(s) for s, _ in ins), 'spill_vgprs': sorted(spill_v)}))
    for o in out:
        print(json.dumps(o))


if __name__ == '__main__':
    main()
