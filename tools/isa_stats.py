"""Per-basic-block instruction histogram of one kernel in a hipcc --save-temps .s file."""
import collections
import re
import sys


def main(path, kernel, top=8):
    s = open(path).read()
    import re as _re
    m = _re.search(r"\n(" + _re.escape(kernel) + r"\w*):", s)  # kernel = a mangled-name prefix
    i = m.start()
    j = s.index(".Lfunc_end", i)  # not the first s_endpgm: a kernel may exit early
    body = s[i:j]
    parts = re.split(r"\n(\.LBB\d+_\d+):", body)
    blocks = [("entry", parts[0])] + [(parts[k], parts[k + 1]) for k in range(1, len(parts), 2)]
    stats = []
    for name, b in blocks:
        ins = [l.strip().split()[0] for l in b.split("\n")
               if l.strip() and not l.strip().startswith((".", ";", "/", "_"))]
        c = collections.Counter(ins)
        stats.append((sum(n for k, n in c.items() if k.startswith("v_")), name, c))
    tot = collections.Counter()
    for _, _, c in stats:
        tot.update(c)
    print("kernel total: valu %d, s_nop %d, scratch %d" % (
        sum(n for k, n in tot.items() if k.startswith("v_")), tot["s_nop"],
        sum(n for k, n in tot.items() if k.startswith("scratch_"))))
    for v, name, c in sorted(stats, reverse=True)[:int(top)]:
        print(name, "valu", v, "s_nop", c["s_nop"], c.most_common(10))


if __name__ == "__main__":
    main(*sys.argv[1:])
