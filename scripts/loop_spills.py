#!/usr/bin/env python3
"""Where the SGPR-spill lane moves sit: for one kernel of snake_kernels.hip's
gfx950 assembly, every loop (a backward branch to an earlier label) with its
instruction count, v_writelane / v_readlane / scratch counts and the source
lines it spans (from -gline-tables-only .loc directives). VERDICT r2 item 2:
count the lane moves inside the draw-round and trace loops before changing them.

    python scripts/loop_spills.py [kernel-substring] [extra hipcc flags...]
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


def main():
    sub = sys.argv[1] if len(sys.argv) > 1 else 'k_autoresetILi4ELb0ELb0E'
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, 'k.s')
        r = subprocess.run(['/opt/rocm/bin/hipcc'] + FLAGS + ['-S', SRC, '-o', asm] + sys.argv[2:],
                           capture_output=True, text=True)
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        text = open(asm).read()
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
