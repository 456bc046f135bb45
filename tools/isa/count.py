"""Instruction classes of a kernel's largest basic block in a hipcc -S file, with an issue-cycle
estimate from DESIGN.md's measured costs (multiply-class and 64-bit VALU ~4 cycles per wave64
instruction, 32-bit logic ~2). Usage: count.py FILE.s KERNEL_PREFIX"""
import collections
import re
import sys

FOUR = ("v_mad_", "v_mul_", "v_lshl_add_u64", "v_ashrrev_i64", "v_lshrrev_b64", "v_lshlrev_b64", "v_mov_b64",
        "v_add_co", "v_addc_co", "v_sub_co", "v_subb_co", "v_add_u64", "v_sub_u64", "v_add3_u32", "v_alignbit")


def blocks(path, kernel):
    s = open(path).read()
    m = re.search(r"\n(" + re.escape(kernel) + r"\w*):", s)
    body = s[m.start():s.index(".Lfunc_end", m.start())]
    parts = re.split(r"\n(\.LBB\d+_\d+):", body)
    out = [("entry", parts[0])] + [(parts[k], parts[k + 1]) for k in range(1, len(parts), 2)]
    res = []
    for name, b in out:
        ins = [l.strip().split()[0] for l in b.split("\n") if l.strip() and not l.strip().startswith((".", ";", "/", "_"))]
        res.append((name, collections.Counter(ins)))
    return res


def main(path, kernel):
    name, c = max(blocks(path, kernel), key=lambda x: sum(n for k, n in x[1].items() if k.startswith("v_")))
    valu = sum(n for k, n in c.items() if k.startswith("v_"))
    four = sum(n for k, n in c.items() if k.startswith(FOUR))
    two = valu - four
    print(f"{kernel} {name}: valu {valu} (4-cycle {four}, 2-cycle {two}), s_nop {c['s_nop']}, "
          f"mad {sum(n for k, n in c.items() if k.startswith('v_mad_'))}, dpp {c['v_mov_b32_dpp']}, "
          f"cndmask {c['v_cndmask_b32_e64'] + c['v_cndmask_b32_e32']}, est. issue cycles {4 * four + 2 * two}")
    print("  ", c.most_common(14))


if __name__ == "__main__":
    for k in sys.argv[2:]:
        main(sys.argv[1], k)
