#!/bin/bash
# Static instruction mix of the tree kernel's time loop by phase (development tool, CPU only):
# the phase profiler's kernel (tools/phase_prof/phase_prof.hip: the product body with s_memtime
# marks between phases) compiled to gfx950 assembly with the product's flags, then counted
# between marks by tools/isa_regions.py.  usage: tools/isa_phase.sh [extra hipcc flags]
set -eu
cd "$(dirname "$0")/.."
C=areafunctionsynthesis_amd/csrc
OUT=${ISA_OUT:-/tmp/isa_phase}
mkdir -p $OUT
/opt/rocm/bin/hipcc -S --cuda-device-only -x hip tools/phase_prof/phase_prof.hip -o $OUT/pp.s --offload-arch=gfx950 \
  -O3 -std=c++17 -fPIC -fno-strict-aliasing -Wno-unknown-pragmas -fno-signed-zeros -mllvm -disable-machine-licm \
  -ffp-contract=fast-honor-pragmas -mllvm -amdgpu-sched-strategy=iterative-ilp -I$C -Iinclude "$@" 2>/dev/null
python3 - "$OUT/pp.s" <<'PY'
import re, sys
L = open(sys.argv[1]).read().split("\n")
s = [i for i, l in enumerate(L) if re.match(r"^_Z\w*tree_prof_kernel\w*:", l)][0]
e = [i for i, l in enumerate(L) if i > s and l.startswith(".Lfunc_end")][0]
body = [l for l in L[s:e]]
open(sys.argv[1] + ".kernel", "w").write("\n".join(body))
PY
python3 tools/isa_regions.py $OUT/pp.s.kernel
