#!/usr/bin/env python3
"""Regenerate tests/golden/known_answers.json (run in the build container).

The fixtures are the reference's own known-answer tests for this path,
reduced to data (inputs per rank + the value the reference test asserts):

* examples/test/coll/allred.c -- 123 MPI_Allreduce cases, every predefined
  (op, type), count 10.  Each case initialises `in` and the expected `sol`
  with C expressions of (i, rank, size).  This script extracts those two
  expressions per case, evaluates them with gcc for communicator sizes 2 and
  4 -- the sizes the reference asserts them at (runtests: np 4; MakeComms in
  examples/test/pt2pt/gcomm.c:24-50 adds the reversed, cartesian (4) and
  odd/even-split (2) communicators) -- and stores the numbers.  (Some
  answers are size-specific, e.g. LXOR of all-ones is 0 only for even p.)
* allredf.f -- the Fortran types (MPI_INTEGER, REAL, DOUBLE_PRECISION,
  COMPLEX, LOGICAL, 2INTEGER, 2REAL, 2DOUBLE_PRECISION), from its closed forms.
* redscat.c (Reduce_scatter SUM INT, recvcounts 1), coll12.c (Reduce MAXLOC /
  Allreduce MINLOC on DOUBLE_INT, TABLE_SIZE 2), redtst.c (BOR: 3|6 == 7),
  shortint.c (Reduce MINLOC SHORT_INT, root 1), scantst.c / coll11.c (Scan SUM
  INT of the rank): closed forms written out below from the checks those
  programs make.

Only the numbers are committed; no reference source text is.  The temporary
C program lives in a temp dir and is deleted.
"""
import json
import os
import re
import subprocess
import tempfile

REF = "/root/reference/examples/test/coll"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "known_answers.json")
SIZES = (2, 4)
COUNT = 10


def allred_cases():
    src = open(os.path.join(REF, "allred.c")).read()
    calls = list(re.finditer(r"MPI_Allreduce\(\s*in,\s*out,\s*count,\s*(MPI_\w+),\s*(MPI_\w+),\s*comm\s*\);", src))
    cases = []
    for m in calls:
        head = src[:m.start()]
        blk = head.rfind("\n{\n")
        body = head[blk:]
        decl = re.search(r"\n(struct\s+\w+\s*\{[^}]*\}|[\w ]+?)\s*\*in,\s*\*out,\s*\*sol;", body)
        loop = body[body.rfind("for (i=0; i<count; i++)"):]
        loop = loop[loop.index("{") + 1: loop.rindex("}")]
        ctype = " ".join(decl.group(1).split())
        cases.append({"type": m.group(1), "op": m.group(2), "ctype": ctype, "init": " ".join(loop.split())})
    return cases


def gen_c(cases):
    out = ["#include <stdio.h>", "#include <math.h>", "int main(void){ int i, count = %d;" % COUNT]
    for k, c in enumerate(cases):
        is_struct = c["ctype"].startswith("struct")
        ctype = c["ctype"]
        out.append("{ %s in_[%d], sol_[%d], out_[%d]; %s *in = in_, *sol = sol_, *out = out_; int rank, size;"
                   % (ctype, COUNT, COUNT, COUNT,
                      ctype if not is_struct else "struct " + ctype.split()[1]))
        out.append("for (size = 2; size <= 4; size += 2) for (rank = 0; rank < size; rank++) {")
        out.append("for (i=0; i<count; i++) { %s }" % c["init"])
        if is_struct:
            out.append('printf("%d %%d %%d", size, rank); for (i=0;i<count;i++) printf(" %%.17g %%d %%.17g %%d",'
                       ' (double)in[i].a, in[i].b, (double)sol[i].a, sol[i].b); printf("\\n");' % k)
        elif "float" in ctype or "double" in ctype:
            out.append('printf("%d %%d %%d", size, rank); for (i=0;i<count;i++) printf(" %%.17g %%.17g",'
                       ' (double)in[i], (double)sol[i]); printf("\\n");' % k)
        else:
            out.append('printf("%d %%d %%d", size, rank); for (i=0;i<count;i++) printf(" %%lld %%lld",'
                       ' (long long)in[i], (long long)sol[i]); printf("\\n");' % k)
        out.append("(void)out; } }")
    out.append("return 0; }")
    return "\n".join(out)


def allredf_cases():
    """examples/test/coll/allredf.f: the Fortran twin of allred.c, MPI_Allreduce
    on MPI_INTEGER / REAL / DOUBLE_PRECISION / COMPLEX / LOGICAL / 2INTEGER /
    2REAL / 2DOUBLE_PRECISION, count 10, i = 1..10.  Its init and solution
    loops are closed forms of (i, rank, size), written out here.  LOGICAL
    words are gfortran's .TRUE. = 1 / .FALSE. = 0 (the MPIR_F_TRUE /
    MPIR_F_FALSE a gfortran build gets); COMPLEX values are [re, im]."""
    out = []
    I = range(1, COUNT + 1)

    def case(t, o, size, fin, fsol, tag=""):
        out.append({"test": "allredf.f" + tag, "coll": "allreduce", "type": t, "op": o, "size": size,
                    "count": COUNT, "inputs": [[fin(r, i) for i in I] for r in range(size)],
                    "expected": [[fsol(i) for i in I]] * size})

    for size in SIZES:
        for t in ("MPI_INTEGER", "MPI_REAL", "MPI_DOUBLE_PRECISION", "MPI_COMPLEX"):
            cx = t == "MPI_COMPLEX"
            val = (lambda x: [x, 0]) if cx else (lambda x: x)
            case(t, "MPI_SUM", size, lambda r, i: val(i), lambda i: val(i * size))
            case(t, "MPI_PROD", size, lambda r, i: val(i), lambda i: val(i ** size))
        for t in ("MPI_INTEGER", "MPI_REAL", "MPI_DOUBLE_PRECISION"):
            case(t, "MPI_MAX", size, lambda r, i: r + i, lambda i: size - 1 + i)
            case(t, "MPI_MIN", size, lambda r, i: r + i, lambda i: i)
        L = "MPI_LOGICAL"
        case(L, "MPI_LOR", size, lambda r, i: int(r % 2 == 1), lambda i: int(size > 1), "(0)")
        case(L, "MPI_LOR", size, lambda r, i: 0, lambda i: 0, "(1)")
        case(L, "MPI_LXOR", size, lambda r, i: int(r == 1), lambda i: int(size > 1), "(0)")
        case(L, "MPI_LXOR", size, lambda r, i: 0, lambda i: 0, "(1)")
        case(L, "MPI_LXOR", size, lambda r, i: 1, lambda i: int(size % 2 != 0), "(2)")
        case(L, "MPI_LAND", size, lambda r, i: int(r % 2 == 1), lambda i: 0, "(0)")
        case(L, "MPI_LAND", size, lambda r, i: 1, lambda i: 1, "(1)")
        N = "MPI_INTEGER"
        case(N, "MPI_BOR", size, lambda r, i: r % 4, lambda i: size - 1 if size < 3 else 3)
        case(N, "MPI_BAND", size, lambda r, i: i if r == size - 1 else -1, lambda i: i, "(1)")
        case(N, "MPI_BAND", size, lambda r, i: i if r == size - 1 else 0, lambda i: 0, "(0)")
        case(N, "MPI_BXOR", size, lambda r, i: 240 if r == 1 else 0, lambda i: 240 if size > 1 else 0, "(1)")
        case(N, "MPI_BXOR", size, lambda r, i: 0, lambda i: 0, "(0)")
        case(N, "MPI_BXOR", size, lambda r, i: -1, lambda i: 0 if size % 2 == 0 else -1, "(1-0)")
        for t in ("MPI_2INTEGER", "MPI_2REAL", "MPI_2DOUBLE_PRECISION"):
            case(t, "MPI_MAXLOC", size, lambda r, i: [r + i, r], lambda i: [size - 1 + i, size - 1])
            case(t, "MPI_MINLOC", size, lambda r, i: [r + i, r], lambda i: [i, 0])
    return out


def num(tok, is_float):
    return float(tok) if is_float else int(tok)


def main():
    cases = allred_cases()
    with tempfile.TemporaryDirectory() as td:
        cfile, exe = os.path.join(td, "ka.c"), os.path.join(td, "ka")
        with open(cfile, "w") as f:
            f.write(gen_c(cases))
        subprocess.check_call(["gcc", "-O0", "-w", "-o", exe, cfile, "-lm"])
        lines = subprocess.check_output([exe]).decode().split("\n")
    for c in cases:
        c["sizes"] = {}
    for line in lines:
        if not line.strip():
            continue
        t = line.split()
        k, size, rank = int(t[0]), int(t[1]), int(t[2])
        c = cases[k]
        is_struct = c["ctype"].startswith("struct")
        is_float = ("float" in c["ctype"] or "double" in c["ctype"])
        vals = t[3:]
        ent = c["sizes"].setdefault(str(size), {"inputs": [None] * size, "expected": None})
        if is_struct:
            vf = "float" in c["ctype"].split("{")[1].split(";")[0] or "double" in c["ctype"].split("{")[1].split(";")[0]
            ins = [[num(vals[4 * i], vf), int(vals[4 * i + 1])] for i in range(COUNT)]
            sol = [[num(vals[4 * i + 2], vf), int(vals[4 * i + 3])] for i in range(COUNT)]
        else:
            ins = [num(vals[2 * i], is_float) for i in range(COUNT)]
            sol = [num(vals[2 * i + 1], is_float) for i in range(COUNT)]
        ent["inputs"][rank] = ins
        if ent["expected"] is None:
            ent["expected"] = sol
        assert ent["expected"] == sol, "sol must not depend on rank"
    for c in cases:
        del c["init"]

    extra = []
    # redscat.c: sendbuf[i] = rank + i, recvcounts 1 -> recv = size*rank + size(size-1)/2
    for size in range(1, 9):
        extra.append({"test": "redscat.c", "coll": "reduce_scatter", "type": "MPI_INT", "op": "MPI_SUM",
                      "size": size, "recvcnts": [1] * size,
                      "inputs": [[r + i for i in range(size)] for r in range(size)],
                      "expected": [[size * r + (size - 1) * size // 2] for r in range(size)]})
    # redtst.c: value = rank == 0 ? 3 : 6; Allreduce BOR -> 7 (size >= 2)
    for size in range(2, 9):
        extra.append({"test": "redtst.c", "coll": "allreduce", "type": "MPI_INT", "op": "MPI_BOR", "size": size,
                      "count": 1, "inputs": [[3 if r == 0 else 6] for r in range(size)],
                      "expected": [[7] for _ in range(size)]})
    # coll12.c: a[i] = 0 for i < rank else rank+1 (MAXLOC, Reduce root 0) and
    # -(rank+1) (MINLOC, Allreduce), loc = rank; checks out[i].b == rank when
    # i % size == rank.  Full answers follow from the MAXLOC/MINLOC tie rule.
    for size in range(1, 9):
        n = 2
        ins_max = [[[float(r + 1) if i >= r else 0.0, r] for i in range(n)] for r in range(size)]
        ins_min = [[[-float(r + 1) if i >= r else 0.0, r] for i in range(n)] for r in range(size)]
        exp_max = [max(((v, -loc) for v, loc in (ins_max[r][i] for r in range(size))))
                   for i in range(n)]
        exp_max = [[v, -nl] for v, nl in exp_max]
        exp_min = [min(((v, loc) for v, loc in (ins_min[r][i] for r in range(size)))) for i in range(n)]
        exp_min = [[v, loc] for v, loc in exp_min]
        extra.append({"test": "coll12.c", "coll": "reduce", "root": 0, "type": "MPI_DOUBLE_INT",
                      "op": "MPI_MAXLOC", "size": size, "count": n, "inputs": ins_max, "expected_root": exp_max})
        extra.append({"test": "coll12.c", "coll": "allreduce", "type": "MPI_DOUBLE_INT", "op": "MPI_MINLOC",
                      "size": size, "count": n, "inputs": ins_min, "expected": [exp_min] * size})
    # shortint.c: s[i] = (rank + i, rank); Reduce MINLOC root 1 -> (i, 0)
    for size in range(2, 9):
        extra.append({"test": "shortint.c", "coll": "reduce", "root": 1, "type": "MPI_SHORT_INT",
                      "op": "MPI_MINLOC", "size": size, "count": 10,
                      "inputs": [[[r + i, r] for i in range(10)] for r in range(size)],
                      "expected_root": [[i, 0] for i in range(10)]})

    # scantst.c / coll11.c: data = rank, MPI_Scan SUM INT -> sum_{i<=rank} i
    for size in range(1, 9):
        extra.append({"test": "scantst.c", "coll": "scan", "type": "MPI_INT", "op": "MPI_SUM", "size": size,
                      "count": 1, "inputs": [[r] for r in range(size)],
                      "expected": [[r * (r + 1) // 2] for r in range(size)]})

    extra += allredf_cases()

    doc = {"generated_by": "tests/golden/gen_known_answers.py",
           "source": "reference examples/test/coll/{allred,redscat,coll12,redtst,shortint,scantst}.c, allredf.f",
           "allred": {"count": COUNT, "sizes": list(SIZES), "cases": cases},
           "other": extra}
    with open(OUT, "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print("wrote %s: %d allred cases, %d other" % (OUT, len(cases), len(extra)))


if __name__ == "__main__":
    main()
