"""Load tests/golden/known_answers.json into per-rank numpy buffers."""
import json
import os

import numpy as np

import importlib

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "golden", "known_answers.json")


def mvx():
    return importlib.import_module("mvapich-cce_amd")


def load():
    with open(PATH) as f:
        return json.load(f)


def handle(name):
    return getattr(mvx(), name)


def np_type(type_name):
    return mvx().NP_DTYPE[handle(type_name)]


def to_array(values, type_name):
    dt = np_type(type_name)
    a = np.zeros(len(values), dt)
    if dt.names:
        a["v"] = [v[0] for v in values]
        a["l"] = [v[1] for v in values]
    elif dt.kind == "c":   # [re, im]
        a[:] = [complex(v[0], v[1]) for v in values]
    elif dt.kind == "u":   # the generator prints unsigned values as long long
        a[:] = [int(v) % (1 << (8 * dt.itemsize)) for v in values]
    else:
        a[:] = values
    return a


def equal(got, expected_arr):
    if expected_arr.dtype.names:
        return bool(np.array_equal(got["v"], expected_arr["v"]) and np.array_equal(got["l"], expected_arr["l"]))
    return bool(np.array_equal(got, expected_arr))


def allred_items():
    """(id, type, op, size, inputs[rank] arrays, expected array)"""
    d = load()
    for k, c in enumerate(d["allred"]["cases"]):
        for size, ent in c["sizes"].items():
            yield (k, c["type"], c["op"], int(size), [to_array(x, c["type"]) for x in ent["inputs"]],
                   to_array(ent["expected"], c["type"]))
