"""The oracle (oracle/chksum_oracle.c) pinned against the reference's golden vectors.

Fixtures: tests/golden/*.json, produced by tests/golden/make_golden.py from the
reference's own Chksum.h compiled in place. Plus SURVEY.md 8(c)'s known answers (taken by
the survey with the reference itself) hard-coded here as an independent pin, and the
reference test's own known answer (tests/ip_chksum_test.cpp:45-62: 0x00FF).
"""
import numpy as np

from conftest import chain_to_chunks
from golden_data import mt19937_64_bytes

# bytes = low 8 bits of std::mt19937_64(42) outputs, prefix of length L
SURVEY_KAT = {0: (0x0000, 0xFFFF), 1: (0xD600, 0x29FF), 2: (0xD6A8, 0x2957),
              3: (0xE0A8, 0x1F57), 20: (0x550C, 0xAAF3), 64: (0xCA82, 0x357D),
              65: (0x5183, 0xAE7C), 1499: (0xD03B, 0x2FC4), 1500: (0xD04C, 0x2FB3),
              9000: (0x78F6, 0x8709)}


def test_survey_known_answers(oracle):
    data = mt19937_64_bytes(42, 9000)
    for ln, (inv, fin) in SURVEY_KAT.items():
        assert oracle.inverted(data, 0, ln) == inv, ln
        assert oracle.final(data, 0, ln) == fin, ln


def test_fixture_known_answers_match_survey(golden):
    got = {ln: (inv, fin) for ln, inv, fin in golden["flat"]["mt19937_64_seed42"]}
    assert got == SURVEY_KAT


def test_flat_cases(oracle, golden):
    b = golden["blob"]
    bad = [(o, l) for o, l, inv, fin in golden["flat"]["flat"]
           if oracle.inverted(b, o, l) != inv or oracle.final(b, o, l) != fin]
    assert not bad, bad[:10]


def test_zero_representation(oracle):
    # 0x0000 only for all-zero input; nonzero input with sum = 0 mod 0xFFFF -> 0xFFFF
    z = np.zeros(1501, dtype=np.uint8)
    f = np.full(1500, 0xFF, dtype=np.uint8)
    assert oracle.inverted(z, 0, 1501) == 0
    assert oracle.inverted(f, 0, 1500) == 0xFFFF
    assert oracle.inverted(z, 0, 0) == 0


def test_reference_test_kat_chain(oracle, golden):
    case = golden["chain"]["chains"][0]
    assert len(case["chunks"]) == 512 and case["chksum"] == 0x00FF
    assert oracle.chain(case["state"], golden["blob"], chain_to_chunks(case)) == 0x00FF


def test_chain_cases(oracle, golden):
    b = golden["blob"]
    bad = []
    for case in golden["chain"]["chains"]:
        got = oracle.chain(case["state"], b, chain_to_chunks(case))
        if got != case["chksum"]:
            bad.append(case)
    assert not bad, bad[:3]


def test_batch_fixtures(oracle, golden):
    from aipstack_amd import synth
    bc = golden["batch"]
    m = bc["mixed_csr"]
    buf, off = synth.mixed_batch(m["n"], m["data_seed"], m["len_seed"])
    assert int(off[-1]) == m["total_bytes"]
    assert oracle.batch_csr(buf, off).tolist() == m["inverted"]
    for name in ("strided_1500", "strided_9000"):
        c = bc[name]
        b = synth.random_bytes(c["data_seed"], c["stride"] * c["n"])
        assert oracle.batch_strided(b, c["stride"], c["len"], c["n"]).tolist() == c["inverted"]
