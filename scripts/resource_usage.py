#!/usr/bin/env python3
"""Per-kernel register / spill / scratch / occupancy table of snake_kernels.hip
(hipcc -Rpass-analysis=kernel-resource-usage), one JSON object per kernel.

    python scripts/resource_usage.py [extra hipcc flags...]
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'marl-snake_amd', 'csrc', 'snake_kernels.hip')


def main():
    cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-ffp-contract=off', '--offload-arch=gfx950',
           '-mllvm', '-amdgpu-atomic-optimizer-strategy=None', '--cuda-device-only', '-c',
           '-Rpass-analysis=kernel-resource-usage', SRC, '-o', os.devnull] + sys.argv[1:]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r'remark: (.*?): (.*?) \[-Rpass', line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == 'Function Name':
            cur = {'kernel': re.sub(r'^_ZN5snake', '', v)[:40]}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    keep = ('TotalSGPRs', 'VGPRs', 'SGPRs Spill', 'VGPRs Spill', 'ScratchSize [bytes/lane]', 'Occupancy [waves/SIMD]')
    for r in rows:
        print(json.dumps({'kernel': r['kernel'], **{k: r.get(k) for k in keep}}))


if __name__ == '__main__':
    main()
