#!/usr/bin/env python3
"""Writes tests/golden/type_known_answers.json: the datatype bounds the
reference's own tests assert (examples/test/pt2pt/*.c), as constructor
sequences plus the expected values -- transcribed from those tests (each
case cites the file and the values it checks).  Only numbers and handle
names are stored; no reference source.

  python tests/golden/gen_type_answers.py
"""
import json
import os

LB_INT_UB = {"ctor": "struct", "count": 3, "blocklens": [1, 1, 1], "indices": [-3, 0, 6],
             "types": ["MPI_LB", "MPI_INT", "MPI_UB"]}

CASES = [
    {"test": "typeub.c", "checks": "extent(type1) == 5*sizeof(int); extent(type2) == 16; extent(type3) == 16 "
                                    "(an MPI_UB buried in a struct member is found)",
     "steps": [
         {"name": "type1", "ctor": "vector", "count": 2, "blocklen": 1, "stride": 4, "old": "MPI_INT"},
         {"name": "type2", "ctor": "struct", "count": 2, "blocklens": [1, 1], "indices": [0, 16],
          "types": ["type1", "MPI_UB"]},
         {"name": "type3", "ctor": "struct", "count": 2, "blocklens": [1, 1], "indices": [0, 4],
          "types": ["type2", "MPI_UB"]}],
     "expect": {"type1": {"extent": 20}, "type2": {"extent": 16}, "type3": {"extent": 16}}},
    {"test": "typeub2.c", "checks": "lb/ub/extent of an explicit {LB -3, INT 0, UB 6} struct, its contiguous(2) "
                                     "and the same as a 2-member struct",
     "steps": [
         dict(name="dt1", **LB_INT_UB),
         {"name": "dt2", "ctor": "contiguous", "count": 2, "old": "dt1"},
         {"name": "dt3", "ctor": "struct", "count": 2, "blocklens": [1, 1], "indices": [0, 9],
          "types": ["dt1", "dt1"]}],
     "expect": {"dt1": {"lb": -3, "ub": 6, "extent": 9}, "dt2": {"lb": -3, "ub": 15, "extent": 18},
                "dt3": {"lb": -3, "ub": 15, "extent": 18}}},
    {"test": "typeub3.c", "checks": "UB / LB taken from the greatest / least instance in hindexed, indexed, "
                                     "hvector and vector",
     "steps": [
         dict(name="dt1", **LB_INT_UB),
         {"name": "dt2", "ctor": "hindexed", "count": 2, "blocklens": [1, 1], "indices": [-4, 7], "old": "dt1"},
         {"name": "dt3", "ctor": "indexed", "count": 2, "blocklens": [1, 1], "indices": [-4, 7], "old": "dt1"},
         {"name": "dt4", "ctor": "hvector", "count": 2, "blocklen": 1, "stride": 14, "old": "dt1"},
         {"name": "dt5", "ctor": "vector", "count": 2, "blocklen": 1, "stride": 14, "old": "dt1"}],
     "expect": {"dt2": {"lb": -7, "ub": 13, "extent": 20}, "dt3": {"lb": -39, "ub": 69, "extent": 108},
                "dt4": {"lb": -3, "ub": 20, "extent": 23}, "dt5": {"lb": -3, "ub": 132, "extent": 135}}},
    {"test": "typelb.c", "checks": "lb == 4, ub == 5, extent == 1 of an hindexed over an hindexed of MPI_BYTE",
     "steps": [
         {"name": "tmp", "ctor": "hindexed", "count": 1, "blocklens": [1], "indices": [3], "old": "MPI_BYTE"},
         {"name": "newtype", "ctor": "hindexed", "count": 1, "blocklens": [1], "indices": [1], "old": "tmp"}],
     "expect": {"newtype": {"lb": 4, "ub": 5, "extent": 1}}},
    {"test": "structlb.c", "checks": "size 1, lb 2, ub 3, extent 1 of a struct over {BYTE at 1, UB at 2}",
     "steps": [
         {"name": "tmptype", "ctor": "struct", "count": 2, "blocklens": [1, 1], "indices": [1, 2],
          "types": ["MPI_BYTE", "MPI_UB"]},
         {"name": "newtype", "ctor": "struct", "count": 1, "blocklens": [1], "indices": [1], "types": ["tmptype"]}],
     "expect": {"newtype": {"size": 1, "lb": 2, "ub": 3, "extent": 1}}},
    {"test": "dataalign.c", "checks": "extent of struct {int; char} == sizeof(struct a) (8 on x86-64: the struct "
                                       "is padded to its largest member)",
     "steps": [
         {"name": "str", "ctor": "struct", "count": 2, "blocklens": [1, 1], "indices": [0, 4],
          "types": ["MPI_INT", "MPI_CHAR"]}],
     "expect": {"str": {"extent": 8}}},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "type_known_answers.json")
    with open(out, "w") as f:
        json.dump({"generated_by": "tests/golden/gen_type_answers.py",
                   "source": "reference examples/test/pt2pt/{typeub,typeub2,typeub3,typelb,structlb,dataalign}.c",
                   "cases": CASES}, f, indent=1)
    print(out)
