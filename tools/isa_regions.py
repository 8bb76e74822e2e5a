"""Static instruction mix of a disassembled kernel between s_memtime markers (development tool).

usage: python tools/isa_regions.py kernel.s
(kernel.s: llvm-objdump -d output of one kernel, e.g. the phase profiler's tree_prof_kernel)
"""
import sys


def main():
    lines = open(sys.argv[1]).read().split("\n")
    marks = [i for i, l in enumerate(lines) if "s_memtime" in l]
    marks = [0] + marks + [len(lines)]
    for a, b in zip(marks, marks[1:]):
        seg = [l.split()[0] for l in lines[a:b] if l.startswith("\t") and l.split()]

        def cnt(p):
            return sum(1 for x in seg if p(x))

        print(f"lines {a:5d}-{b:5d}: instr {len(seg):5d} valu {cnt(lambda x: x.startswith('v_')):5d} "
              f"f64 {cnt(lambda x: '_f64' in x):4d} ds {cnt(lambda x: x.startswith('ds_')):4d} "
              f"accvgpr {cnt(lambda x: 'accvgpr' in x):4d} rw-lane {cnt(lambda x: 'lane_b32' in x):4d} "
              f"dpp {cnt(lambda x: 'dpp' in x):3d} br {cnt(lambda x: x.startswith('s_cbranch') or x == 's_branch'):3d} "
              f"waitcnt {cnt(lambda x: x == 's_waitcnt'):4d}")


if __name__ == "__main__":
    main()
