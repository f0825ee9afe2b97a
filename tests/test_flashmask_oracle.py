"""CPU checks of the FlashMask restatement (oracle/flashmask_ref.py): vectorised form against the
reference-ordered loop form, plus hand-derived known answers."""
import numpy as np
import pytest

from oracle.flashmask_ref import document_lts, flashmask_keep, flashmask_keep_loops


@pytest.mark.parametrize("mode", ["causal", "causal_end", "bidir2", "bidir4"])
def test_vectorised_matches_loops(mode):
    rng = np.random.default_rng(3)
    b, hm, sq, sk = 2, 2, 13, 11
    draw = lambda: rng.integers(0, sq + 3, size=(b, hm, sk)).astype(np.int32)  # noqa: E731
    lts, lte, uts, ute = draw(), draw(), draw(), draw()
    causal = mode.startswith("causal")
    kw = {}
    if mode == "causal_end":
        kw = dict(lte=lte)
    elif mode == "bidir2":
        kw = dict(ute=ute)
    elif mode == "bidir4":
        kw = dict(lte=lte, uts=uts, ute=ute)
    np.testing.assert_array_equal(flashmask_keep(lts, sq, causal, **kw),
                                  flashmask_keep_loops(lts, sq, causal, **kw))


def test_negative_bounds_compare_unsigned():
    lts = np.full((1, 1, 4), -1, dtype=np.int32)   # 0xffffffff: never reached -> nothing masked
    keep = flashmask_keep(lts, 4, True)
    np.testing.assert_array_equal(keep[0, 0], np.tril(np.ones((4, 4), dtype=bool)))
    np.testing.assert_array_equal(keep, flashmask_keep_loops(lts, 4, True))


def test_causal_document_mask_is_block_diagonal():
    docs = [3, 5, 2]
    sq = sum(docs)
    lts = document_lts(docs, sq)[None, None]
    keep = flashmask_keep(lts, sq, True)[0, 0]
    doc = np.repeat(np.arange(len(docs)), docs)
    want = (doc[:, None] == doc[None, :]) & np.tril(np.ones((sq, sq), dtype=bool))
    np.testing.assert_array_equal(keep, want)


def test_bidirectional_no_op_and_sliding_band():
    sq = sk = 9
    lts = np.full((1, 1, sk), sq, dtype=np.int32)
    ute = np.zeros((1, 1, sk), dtype=np.int32)
    assert flashmask_keep(lts, sq, False, ute=ute).all()
    # band |q - k| <= 2: rows >= k + 3 masked (LT), rows < k - 2 masked (UT)
    k = np.arange(sk)
    lts = (k + 3)[None, None].astype(np.int32)
    ute = np.maximum(k - 2, 0)[None, None].astype(np.int32)
    keep = flashmask_keep(lts, sq, False, ute=ute)[0, 0]
    q = np.arange(sq)[:, None]
    np.testing.assert_array_equal(keep, np.abs(q - k[None]) <= 2)
