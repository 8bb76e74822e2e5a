"""Count the fp64 operations the reference algorithm performs per audio sample.

The oracle restatement (oracle/afs_oracle.c, the reference's operation order) is compiled to
LLVM IR at -O0 with no fp contraction, so every arithmetic operation written in the source is
one IR instruction.  Each basic block gets a call fc_bb(id) after its phis; the static count of
fp64 instructions per block times the block's execution count is the dynamic count.  The
instrumented IR is then compiled with optimisation (the calls are opaque, so they run exactly
when their blocks would).

python tools/flopcount/instrument.py      -> tools/flopcount/_build/liboracle_fc.so
Counted: fadd fsub fmul fdiv on double, sqrt, transcendental calls (exp pow log log10 cos
sin tan), and separately fcmp / fneg / fabs (not flops).  Measurement tooling, not product.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CLANG = "/opt/rocm/lib/llvm/bin/clang"
KINDS = ["add", "sub", "mul", "div", "sqrt", "transc", "cmp", "neg"]
TRANSC = ("exp", "pow", "log", "log10", "cos", "sin", "tan")

LABEL = re.compile(r"^([A-Za-z0-9_.$]+):(\s|$)")


def classify(line: str):
    s = line.strip()
    if re.search(r"= fadd (\w+ )*double ", s):
        return "add"
    if re.search(r"= fsub (\w+ )*double ", s):
        return "sub"
    if re.search(r"= fmul (\w+ )*double ", s):
        return "mul"
    if re.search(r"= fdiv (\w+ )*double ", s):
        return "div"
    if re.search(r"= fneg (\w+ )*double ", s):
        return "neg"
    if re.search(r"= fcmp \w+ double ", s):
        return "cmp"
    m = re.search(r"call (?:\w+ )*double @(?:llvm\.)?([a-z0-9_]+?)(?:\.f64)?\(", s)
    if m:
        f = m.group(1)
        if f == "sqrt":
            return "sqrt"
        if f in TRANSC:
            return "transc"
    if re.search(r"= fmuladd|@llvm\.fma", s):
        raise SystemExit("contracted multiply-add in the IR: build with -ffp-contract=off")
    return None


def instrument(ll: str):
    out, table, fns = [], [], []
    in_fn = False
    fn = None
    pending = None  # counts of the block being emitted (inserted once its phis are done)
    cur = None

    def open_block():
        nonlocal cur, pending
        cur = [0] * len(KINDS)
        table.append(cur)
        fns.append(fn)
        pending = len(table) - 1

    for line in ll.splitlines():
        if line.startswith("define "):
            m = re.search(r"@([A-Za-z0-9_.$]+)\(", line)
            fn = m.group(1) if m else "?"
            in_fn = True
            out.append(line)
            open_block()
            continue
        if in_fn and line.startswith("}"):
            in_fn = False
            out.append(line)
            continue
        if not in_fn:
            out.append(line)
            continue
        if LABEL.match(line):
            out.append(line)
            open_block()
            continue
        s = line.strip()
        if pending is not None and s and not s.startswith(";") and " = phi " not in s:
            out.append(f"  call void @fc_bb(i32 {pending})")
            pending = None
        k = classify(line)
        if k:
            cur[KINDS.index(k)] += 1
        out.append(line)
    out.append("declare void @fc_bb(i32)")
    return "\n".join(out) + "\n", table, fns


def main() -> None:
    build = os.path.join(HERE, "_build")
    os.makedirs(build, exist_ok=True)
    ll = os.path.join(build, "oracle.ll")
    subprocess.check_call([CLANG, "-O0", "-ffp-contract=off", "-fno-builtin", "-S", "-emit-llvm", "-o", ll,
                           os.path.join(ROOT, "oracle", "afs_oracle.c")])
    text, table, fns = instrument(open(ll).read())
    # the static table with each block's function (count.py splits the counts by function)
    import json
    json.dump({"kinds": KINDS, "ops": table, "fn": fns}, open(os.path.join(build, "fc_blocks.json"), "w"))
    ill = os.path.join(build, "oracle_fc.ll")
    open(ill, "w").write(text)
    rt = os.path.join(build, "fc_table.c")
    with open(rt, "w") as f:
        f.write("#include <stdint.h>\n#include <string.h>\n")
        f.write(f"#define NB {len(table)}\n#define NK {len(KINDS)}\n")
        f.write("static const uint8_t ops[NB][NK] = {\n")
        f.write(",\n".join("{" + ",".join(str(v) for v in row) + "}" for row in table))
        f.write("};\nstatic uint64_t hits[NB];\n")
        f.write("void fc_bb(int32_t id) { ++hits[id]; }\n")
        f.write("void fc_reset(void) { memset(hits, 0, sizeof hits); }\n")
        f.write("int fc_nblocks(void) { return NB; }\n")
        f.write("void fc_hits(uint64_t *out) { memcpy(out, hits, sizeof hits); }\n")
        f.write("void fc_read(uint64_t *out) { for (int k = 0; k < NK; ++k) { out[k] = 0; "
                "for (int b = 0; b < NB; ++b) out[k] += hits[b] * ops[b][k]; } }\n")
    so = os.path.join(build, "liboracle_fc.so")
    subprocess.check_call([CLANG, "-O2", "-fPIC", "-shared", "-o", so, ill, rt, "-lm"])
    print(so, f"({len(table)} blocks)")


if __name__ == "__main__":
    sys.exit(main())
