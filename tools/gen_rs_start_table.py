"""Prints the Aberth start-point table of csrc/rs_math.h (RS_START_RE / RS_START_IM):
cos / sin of 2 pi r / n + 0.4 for n = 1..10, r = 0..n-1 (zero for r >= n), as exact
hexadecimal doubles.  The GPU solver (csrc/ransac.hip real_roots10) and its C twin
(oracle/csrc/ransac_cv.c) both read this one table, so their start points -- and with
them every Aberth iterate -- are the same bits.

    python tools/gen_rs_start_table.py"""
import math


def rows(fn):
    out = []
    for n in range(1, 11):
        vals = [float(fn(6.283185307179586 * r / n + 0.4)).hex() if r < n else "0x0p+0" for r in range(10)]
        out.append("    {" + ", ".join(vals) + "},")
    return "\n".join(out)


if __name__ == "__main__":
    print("RS_CONST double RS_START_RE[10][10] = {\n" + rows(math.cos) + "\n};")
    print("RS_CONST double RS_START_IM[10][10] = {\n" + rows(math.sin) + "\n};")
