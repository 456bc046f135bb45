"""Check tools/f29_bench's dump (radix-2^29 Montgomery ops, R = 2^261) with Python big ints."""
import struct
import sys

P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
RINV = pow(2 ** 261, -1, P)


def val(limbs):
    return sum(((w ^ 0x80000000) - 0x80000000) << (29 * i) for i, w in enumerate(limbs))


def normal(limbs):
    return all(0 <= w < 2 ** 29 for w in limbs[:8]) and abs(val(limbs)) < 2 ** 258


def main(path):
    raw = open(path, "rb").read()
    n = len(raw) // 4 // (16 + 27)
    w = struct.unpack("<%dI" % (len(raw) // 4), raw)
    inp, out = w[:16 * n], w[16 * n:]
    bad = 0
    for t in range(n):
        a = sum(inp[16 * t + i] << (32 * i) for i in range(8))
        b = sum(inp[16 * t + 8 + i] << (32 * i) for i in range(8))
        m, s, d = out[27 * t:27 * t + 9], out[27 * t + 9:27 * t + 18], out[27 * t + 18:27 * t + 27]
        em = a * b * RINV % P
        es = a * a * RINV % P
        ed = (em - es) * 3 * (em + es) * RINV % P
        ok = (val(m) % P == em and val(s) % P == es and val(d) % P == ed and normal(m) and normal(s)
              and normal(d))
        if not ok:
            bad += 1
            if bad < 5:
                print("case", t, hex(a), hex(b), val(m) % P == em, val(s) % P == es, val(d) % P == ed,
                      normal(m), normal(s), normal(d))
    print("f29 check: %d cases, %d bad" % (n, bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
