"""The CPU restatement (oracle/) pinned against the reference tools' own outputs.

tests/golden/*.json.gz were produced by tests/golden/make_golden.py, which runs
/root/reference/tools/1.convert_AG_to_CT.py and 2.extend_gap.py on the same inputs.
"""
import numpy as np
import pytest

from helpers import compare_records, golden_inputs, load_golden
from oracle import oracle


def test_tool1_fuzz_matches_reference():
    g = load_golden("tool1_fuzz.json.gz")
    raw, ref = golden_inputs(g)
    res = oracle.run(raw, ref)
    compare_records(g["tool1"], res.tool1, raw, g["input"], "tool1-fuzz")


def test_tools12_families_match_reference():
    g = load_golden("tool12_families.json.gz")
    raw, ref = golden_inputs(g)
    res = oracle.run(raw, ref)
    compare_records(g["tool1"], res.tool1, raw, g["input"], "tool1-families")
    compare_records(g["tool2"], res.tool2, raw, g["input"], "tool2-families")


def test_tool2_missing_mi_raises_like_reference():
    g = load_golden("tool2_missing_mi.json.gz")
    assert g["tool2_error"] and "does not have MI tag" in g["tool2_error"]
    raw, ref = golden_inputs(g)
    with pytest.raises(oracle.OracleError, match="does not have MI tag"):
        oracle.run(raw, ref)
