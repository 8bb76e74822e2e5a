#!/bin/bash
# Builds the fp32-state variant of the oracle restatement for the precision study
# (tools/fp32_study/study.py): every `double` of the synthesis part of oracle/afs_oracle.c
# -- tube, glottis, noise sources, matrix, solver and state updates, from the rand() section
# to the OneDimAreaFunction section -- becomes `float`, except in the public entry points,
# whose signatures keep the header's double interface (frames in, audio out).  Constants, the
# IIR filters (output Chebyshev, glottal tone, noise shaping) and libm calls stay double: a
# best case for fp32 tube state.
# Output: tools/fp32_study/_build/liboracle_f32.so (git-ignored).
set -eu
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
mkdir -p "$HERE/_build"
SRC="$HERE/_build/afs_oracle_f32.c"
BEGIN=$(grep -n "glibc random_r TYPE_3" "$ROOT/oracle/afs_oracle.c" | head -1 | cut -d: -f1)
END=$(grep -n "OneDimAreaFunction (OneDimAreaFunction.cpp" "$ROOT/oracle/afs_oracle.c" | head -1 | cut -d: -f1)
sed "${BEGIN},${END}s/\bdouble\b/float/g" "$ROOT/oracle/afs_oracle.c" > "$SRC"
for fn in ao_chebyshev ao_fulcher_kent ao_create ao_synthesize_call ao_get_pressures ao_get_currents \
          ao_get_state ao_synthesize_utterance; do
  sed -i -E "/^[a-z_ ]+\**[ *]${fn}\(/,/\{/ s/\bfloat\b/double/g" "$SRC"
done
sed -i "s|#include \"afs_oracle.h\"|#include \"$ROOT/oracle/afs_oracle.h\"|" "$SRC"
gcc -std=c11 -O2 -fPIC -shared -w -o "$HERE/_build/liboracle_f32.so" "$SRC" -lm
echo "$HERE/_build/liboracle_f32.so"
