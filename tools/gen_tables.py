#!/usr/bin/env python3
"""Emit reinforcementlearning_blokus_amd/csrc/orient_table.h.

Restates engine/pieces.py:147-253 (generate_orientations_for_piece) for the 21
shapes of engine/pieces.py:289-356: variants rot0..rot270 (numpy.rot90, counter-
clockwise), then fliplr and its three rotations; a variant whose sorted normalized
offsets were already seen is dropped.  The global orientation id g runs piece-major
(piece 1 first), orientation index ascending: g order == reference list order.

tests/test_tables.py checks the emitted table against tests/golden/pieces.json.
"""
import os

SHAPES = [
    "1", "11", "111", "10|11", "1111", "11|11", "111|010", "10|10|11", "011|110", "110|011",
    "011|110|010", "11111", "10|10|10|11", "10|11|01|01", "11|11|10", "111|010|010", "101|111",
    "100|100|111", "100|110|011", "010|111|010", "10|11|10|10",
]


def rot90(m):
    h, w = len(m), len(m[0])
    return [[m[j][w - 1 - i] for j in range(h)] for i in range(w)]


def fliplr(m):
    return [row[::-1] for row in m]


def orientations():
    table = []
    for pid, s in enumerate(SHAPES, start=1):
        base = [[int(ch) for ch in row] for row in s.split("|")]
        variants = [base]
        for _ in range(3):
            variants.append(rot90(variants[-1]))
        variants.append(fliplr(base))
        for _ in range(3):
            variants.append(rot90(variants[-1]))
        seen = []
        for v in variants:
            cells = sorted((r, c) for r, row in enumerate(v) for c, x in enumerate(row) if x)
            if cells in seen:
                continue
            seen.append(cells)
            table.append((pid, len(seen) - 1, cells, len(v), len(v[0])))
    return table


# stencil term kinds: one cell, a horizontal pair (plane BP = B | B >> 1), a vertical
# pair (plane BV[R] = B[R] | B[R + 1])
KINDS = {"s": 0, "p": 1, "v": 2}
VPAIR = os.environ.get("BK_GEN_VPAIR", "0") == "1"  # measured: 2 waves/SIMD needed, net slower


def _placements(cells):
    cs = set(cells)
    out = []
    for (r, c) in cells:
        out.append(("s", r, c, frozenset([(r, c)])))
        if (r, c + 1) in cs:
            out.append(("p", r, c, frozenset([(r, c), (r, c + 1)])))
        if VPAIR and (r + 1, c) in cs:
            out.append(("v", r, c, frozenset([(r, c), (r + 1, c)])))
    return out


def stencil_terms(cells):
    """Cover an orientation's cells with the fewest singles / horizontal / vertical pairs (overlap
    allowed: the stencil ORs shifted rows, so covering a cell twice is harmless).
    Returns [(kind, d, c), ...] with a column-0 term first (it needs no shift), the
    rest sorted by (d, kind, c)."""
    import itertools
    target = frozenset(cells)
    P = _placements(cells)
    for k in range(1, 6):
        for combo in itertools.combinations(P, k):
            if frozenset().union(*[x[3] for x in combo]) == target:
                terms = sorted(((x[0], x[1], x[2]) for x in combo), key=lambda t: (t[1], t[0], t[2]))
                z = next(i for i, t in enumerate(terms) if t[2] == 0)
                return [terms[z]] + terms[:z] + terms[z + 1:]
    raise AssertionError(cells)


def render_classes(table):
    """Stencil classes.  A class = (height, term sequence [(d, kind)]) -- the static
    shape of the straight-line code that scans it; the column shifts of terms 1.. are
    per-orientation (uniform) operands.  Per orientation 2 words in class order:
    w0 = piece_id | g << 8, w1 = column of term k (k >= 1) at bits 3(k-1).
    BK_CLASS_LIST(X) expands X(i0, i1, height, t0, t1, ...) per class with
    t = d * 4 + kind (KINDS)."""
    classes = {}
    for g, (pid, _o, cells, h, _w) in enumerate(table):
        terms = stencil_terms(cells)
        key = (h, tuple(d * 4 + KINDS[k] for k, d, _c in terms))
        w1 = sum(c << (3 * (j - 1)) for j, (_k, _d, c) in enumerate(terms) if j > 0)
        classes.setdefault(key, []).append((pid | (g << 8), w1))
    order = sorted(classes, key=lambda k: (k[0], len(k[1]), k[1]))
    lines = [f"#define BK_NUM_CLASSES {len(order)}",
             f"#define BK_STENCIL_TERMS {sum(len(k[1]) * len(classes[k]) for k in order)}",
             "#define BK_CLASS_LIST(X) \\"]
    i = 0
    rows = []
    for k in order:
        n = len(classes[k])
        lines.append(f"    X({i}, {i + n}, {k[0]}, {', '.join(str(t) for t in k[1])}) \\")
        rows += classes[k]
        i += n
    lines.append("")
    lines.append("#define BK_CLASS_TABLE_INIT { \\")
    for w0, w1 in rows:
        lines.append(f"    {{{hex(w0)}, {hex(w1)}}}, \\")
    lines.append("}")
    return lines


def render_cell_hash():
    """hash((r, c)) of this CPython (3.10: xxHash-based tuplehash over the int hashes),
    as the 64-bit pattern: the frontier sets' slot order depends on it
    (engine/board.py:70 player_frontiers are sets of (row, col) tuples)."""
    import sys
    assert sys.version_info[:2] == (3, 10), "the reference runs CPython 3.10"
    vals = [hash((r, c)) & (2**64 - 1) for r in range(20) for c in range(20)]
    lines = ["// CPython 3.10 hash((r, c)) for cell r*20+c (frontier set slot order)",
             "#define BK_CELL_HASH_INIT { \\"]
    for i in range(0, 400, 4):
        lines.append("    " + ", ".join(f"{v:#018x}ull" for v in vals[i:i + 4]) + ", \\")
    lines.append("}")
    return lines


def render(table):
    lines = [
        "// Generated by tools/gen_tables.py -- do not edit.",
        "// 91 orientations of the 21 reference pieces (engine/pieces.py:147-356),",
        "// global id g piece-major / orientation-ascending == reference list order.",
        "#pragma once",
        "#include <stdint.h>",
        f"#define BK_NUM_ORIENTS {len(table)}",
        "// info: piece_id | ncells << 8 | height << 16 | width << 24",
        "static const uint32_t kOrientInfoHost[BK_NUM_ORIENTS] = {",
    ]
    for pid, _o, cells, h, w in table:
        lines.append(f"    {pid} | ({len(cells)} << 8) | ({h} << 16) | ({w} << 24),")
    lines.append("};")
    lines.append("// cells: row << 8 | col, sorted (row-major); unused entries 0")
    lines.append("static const uint32_t kOrientCellsHost[BK_NUM_ORIENTS][5] = {")
    for _pid, _o, cells, _h, _w in table:
        vals = [f"({r} << 8) | {c}" for r, c in cells] + ["0"] * (5 - len(cells))
        lines.append("    {" + ", ".join(vals) + "},")
    lines.append("};")
    lines.append("// orientation index within the piece (Move.orientation)")
    lines.append("static const uint8_t kOrientIndexHost[BK_NUM_ORIENTS] = {")
    lines.append("    " + ", ".join(str(o) for _p, o, _c, _h, _w in table))
    lines.append("};")
    lines.append("// initializer lists for __constant__ device copies")
    lines.append("#define BK_ORIENT_INFO_INIT { \\")
    for pid, _o, cells, h, w in table:
        lines.append(f"    {pid} | ({len(cells)} << 8) | ({h} << 16) | ({w} << 24), \\")
    lines.append("}")
    lines.append("#define BK_ORIENT_CELLS_INIT { \\")
    for _pid, _o, cells, _h, _w in table:
        vals = [f"({r} << 8) | {c}" for r, c in cells] + ["0"] * (5 - len(cells))
        lines.append("    {" + ", ".join(vals) + "}, \\")
    lines.append("}")
    lines.append("// rows: per orientation and piece row d (0..4): ncells << 16 | col_j << 3j")
    lines.append("#define BK_ORIENT_ROWS_INIT { \\")
    for _pid, _o, cells, _h, _w in table:
        words = []
        for d in range(5):
            cols = [c for r, c in cells if r == d]
            w = (len(cols) << 16) | sum(c << (3 * j) for j, c in enumerate(cols))
            words.append(hex(w))
        lines.append("    {" + ", ".join(words) + "}, \\")
    lines.append("}")
    lines += render_classes(table)
    lines += render_cell_hash()
    return "\n".join(lines) + "\n"


def main():
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                       "reinforcementlearning_blokus_amd", "csrc", "orient_table.h")
    with open(out, "w") as f:
        f.write(render(orientations()))
    print("wrote", os.path.normpath(out))


if __name__ == "__main__":
    main()
