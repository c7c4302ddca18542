#!/usr/bin/env python3
"""Static instruction counts per kernel of snake_kernels.hip (gfx950 assembly):
SGPR-spill lane moves (v_writelane / v_readlane: the compiler spills SGPRs into
VGPR lanes), scratch accesses (VGPR spills), and the total, merged with the
resource-usage remarks. One JSON object per kernel.

    python scripts/isa_counts.py [extra hipcc flags...] > profiles/r03_isa_counts.jsonl
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
         '-amdgpu-atomic-optimizer-strategy=None', '--cuda-device-only']


def demangle(name):
    r = subprocess.run(['c++filt', name], capture_output=True, text=True)
    return r.stdout.strip().replace('snake::', '') or name


def main():
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, 'k.s')
        r = subprocess.run(['/opt/rocm/bin/hipcc'] + FLAGS + ['-S', '-Rpass-analysis=kernel-resource-usage', SRC,
                            '-o', asm] + sys.argv[1:], capture_output=True, text=True)
        if r.returncode:
            sys.exit(r.stderr[-2000:])
        text = open(asm).read()
    usage, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r'remark: (.*?): (.*?) \[-Rpass', line)
        if m and m.group(1).strip() == 'Function Name':
            cur = m.group(2).strip()
            usage[cur] = {}
        elif m and cur:
            usage[cur][m.group(1).strip()] = m.group(2).strip()
    # kernel bodies: from "<name>:" to its ".Lfunc_end"
    for m in re.finditer(r'^(_Z\w+):[^\n]*$(.*?)^\.Lfunc_end', text, re.S | re.M):
        name, body = m.group(1), m.group(2)
        ins = [ln.strip() for ln in body.splitlines()
               if ln.startswith('\t') and not ln.strip().startswith(('.', ';')) and ln.strip()]
        u = usage.get(name, {})
        if not u:
            continue
        print(json.dumps({
            'kernel': demangle(name),
            'instructions': len(ins),
            'v_writelane': sum(i.startswith('v_writelane') for i in ins),
            'v_readlane': sum(i.startswith('v_readlane') for i in ins),
            'scratch_ops': sum(i.startswith(('scratch_', 'buffer_store', 'buffer_load')) for i in ins),
            'SGPRs Spill': u.get('SGPRs Spill'), 'VGPRs': u.get('VGPRs'), 'VGPRs Spill': u.get('VGPRs Spill'),
            'ScratchSize': u.get('ScratchSize [bytes/lane]'), 'Occupancy': u.get('Occupancy [waves/SIMD]'),
        }))


if __name__ == '__main__':
    main()
