"""CPU check of the stuffing tail's word fetch (k_count_ff / k_write `group_values`) through its
lane-level model (tests/tail_model.py): every segment word equals the concatenated chunk bits
with the 1-bit byte padding, and no slot load leaves the words k_encode wrote (the chunk's
ceil(L / 32) words, or the next chunk's first word)."""
import numpy as np
import pytest

from tail_model import G, R, Seg, segment_words


def _layouts():
    rng = np.random.default_rng(7)
    yield "one short chunk", [12]
    yield "short last chunk inside the previous chunk's last word", [1000, 12]
    yield "short last chunk ending a word", [1000, 24]
    yield "short last chunk at a word start", [992, 7]
    yield "word-aligned chunks", [1024] * 5
    yield "two groups, short tail", [900] * G + [300, 5]
    yield "group boundary chunk in one word", [256] * (G - 1) + [260, 3]
    for t in range(12):
        n = int(rng.integers(1, 3 * G))
        L = rng.integers(256, 4000, n)
        if rng.random() < 0.5:
            L[-1] = int(rng.integers(1, 40))
        if rng.random() < 0.3:
            L[: n // 2] = rng.integers(256, 300, n // 2)
        yield f"random {t}", L.tolist()
    yield "long chunks (many rounds)", [64 * 1664] * 3 + [4]


@pytest.mark.parametrize("name,lengths", list(_layouts()))
def test_group_values_model(name, lengths):
    seg = Seg(lengths, np.random.default_rng(len(lengths)))
    got = segment_words(seg)
    exp = seg.expected_words()
    assert sorted(got) == list(range(len(exp))), "words missing or extra"
    bad = [k for k in got if got[k] != int(exp[k])]
    assert not bad, f"{len(bad)} words differ, first {bad[0]}: {got[bad[0]]:08x} != {int(exp[bad[0]]):08x}"
    oob = [t for t in seg.touched if not t[2]]
    assert not oob, f"loads outside the written words: {oob[:5]}"
    assert R >= 1
