#!/bin/bash
# Register budget of the search kernels in a built object (default: the main build):
#   tools/kernel_regs.sh [path/to/hastar_kernels.o]
# prints name, VGPRs, SGPRs, SGPR/VGPR spill counts and scratch bytes from the code object notes.
set -e
OBJ=${1:-path_planning_pkg_amd/lib/hastar_kernels.o}
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy -O binary --only-section=.hip_fatbin "$OBJ" $T/fb.bin
$B/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$B/llvm-readelf --notes $T/k.co | python3 -c "
import sys, re
cur = {}
rows = []
for line in sys.stdin:
    m = re.match(r'\s+\.(name|sgpr_count|vgpr_count|agpr_count|sgpr_spill_count|vgpr_spill_count|private_segment_fixed_size|group_segment_fixed_size):\s+(\S+)', line)
    if not m: continue
    k, v = m.groups()
    if k == 'name': cur = {'name': v}; rows.append(cur)
    else: cur[k] = v
for r in rows:
    if (('search' in r['name'] and 'k_' not in r['name']) or 'reloc' in r['name']):
        print(r['name'][:60], 'vgpr', r.get('vgpr_count'), 'agpr', r.get('agpr_count'), 'sgpr', r.get('sgpr_count'), 'sgpr_spill', r.get('sgpr_spill_count'),
              'vgpr_spill', r.get('vgpr_spill_count'), 'scratch', r.get('private_segment_fixed_size'), 'lds', r.get('group_segment_fixed_size'))
"
rm -rf $T
