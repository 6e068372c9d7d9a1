"""The reference's exported helpers (SURVEY §8(b) "helpers keep the ABI") against golden
vectors the reference itself produced (tests/golden/helpers.npz, gen_golden.py
gen_helpers):

  nybble_compression.c  byte_to_context :517, initialize_dictionary :546,
                        update_context :665, compress_byte_index :819, decompress_nybble :643
                        -> libdc_nybble.so (host: one byte of the caller's table per call)
  n_ary_huffman.c       setup_nodes :773, find_compressed_data_size :2466 (host),
                        generate_huffman_tree :868, summarize_tree_with_lengths :1033 (GPU)
"""
import ctypes as C
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAXSYM = 258


class Node(C.Structure):   # struct node (include/dc_huffman.h)
    _fields_ = [("leaf", C.c_bool), ("count", C.c_int), ("left_index", C.c_int), ("right_index", C.c_int),
                ("leaf_value", C.c_int), ("parent_index", C.c_int), ("volume", C.c_int)]


FIELDS = ("leaf", "count", "left_index", "right_index", "leaf_value", "parent_index")


class CtxTable(C.Structure):   # context_table_type (include/dc_nybble.h)
    _fields_ = [("letter", (C.c_char * 8) * 16), ("times_used_directly", C.c_int * 16)]


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(G, "helpers.npz"), allow_pickle=False)


@pytest.fixture(scope="module")
def nyb():
    from data_compression_amd._lib import load
    L = load("libdc_nybble.so")
    L.byte_to_context.argtypes = [C.c_char]
    L.byte_to_context.restype = C.c_int
    L.initialize_dictionary.argtypes = [C.POINTER(CtxTable)]
    L.update_context.argtypes = [C.POINTER(CtxTable), C.c_char, C.c_char]
    L.update_context.restype = C.c_int
    L.compress_byte_index.argtypes = [C.POINTER(CtxTable), C.c_int, C.c_char_p, C.c_char_p]
    L.compress_byte_index.restype = C.c_int
    L.decompress_nybble.argtypes = [CtxTable, C.c_char, C.c_char, C.c_char_p]
    L.decompress_nybble.restype = C.c_int
    return L


@pytest.fixture(scope="module")
def huf():
    from data_compression_amd._lib import load
    L = load("libdc_huffman.so")
    L.setup_nodes.argtypes = [C.c_int, C.POINTER(Node), C.c_int, C.POINTER(C.c_int)]
    L.generate_huffman_tree.argtypes = [C.c_int, C.POINTER(Node), C.c_int, C.c_int]
    L.summarize_tree_with_lengths.argtypes = [C.c_int, C.POINTER(Node), C.c_int, C.POINTER(C.c_int), C.c_int]
    L.find_compressed_data_size.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int]
    L.find_compressed_data_size.restype = C.c_int
    return L


def _nodes(lst):
    return np.array([[int(getattr(nd, f)) for f in FIELDS] for nd in lst], dtype=np.int64)


# ---------------------------------------------------------------- nybble helpers (host)
def test_byte_to_context_and_dictionary(gold, nyb):
    got = [nyb.byte_to_context(bytes([b])) for b in range(256)]
    assert np.array_equal(np.array(got, np.int32), gold["b2c"])
    t = CtxTable()
    nyb.initialize_dictionary(C.byref(t))
    assert bytes(t) == gold["init_table"].tobytes()


def test_update_context_sequence(gold, nyb):
    t = CtxTable()
    nyb.initialize_dictionary(C.byref(t))
    text = gold["upd_text"]
    snaps = gold["upd_snaps"]
    k = 0
    for i in range(1, text.size):
        assert nyb.update_context(C.byref(t), bytes([int(text[i - 1])]), bytes([int(text[i])])) == 0
        if i % 100 == 0:
            assert bytes(t) == snaps[k].tobytes(), i
            k += 1
    assert k == len(snaps)


def test_compress_byte_index_and_decompress_nybble(gold, nyb):
    snaps = gold["upd_snaps"]
    for snap, off, prev, cur, d0, d1, r, e0, e1 in gold["cbi"]:
        tb = CtxTable.from_buffer_copy(snaps[snap].tobytes())
        src = C.create_string_buffer(bytes([int(prev), int(cur), 0]), 3)
        dst = C.create_string_buffer(bytes([int(d0), int(d1), 0]), 3)
        got = nyb.compress_byte_index(C.byref(tb), int(off), C.cast(C.addressof(src) + 1, C.c_char_p), dst)
        assert (got, dst.raw[0], dst.raw[1]) == (r, e0, e1)
    for snap, prev, nybv, nxt, r, e in gold["dnyb"]:
        dd = C.create_string_buffer(bytes([int(prev), 0x5A, 0]), 3)
        got = nyb.decompress_nybble(CtxTable.from_buffer_copy(snaps[snap].tobytes()), bytes([int(nybv)]),
                                    bytes([int(nxt)]), C.cast(C.addressof(dd) + 1, C.c_char_p))
        assert (got, dd.raw[1]) == (r, e)


# ---------------------------------------------------------------- Huffman helpers
def test_setup_nodes_and_data_size(gold, huf):
    for f, setup, L, size in zip(gold["tree_freq"], gold["tree_setup"], gold["tree_lengths"], gold["tree_size"]):
        fr = (C.c_int * (MAXSYM + 1))(*[int(v) for v in f])
        lst = (Node * (2 * MAXSYM))()
        for nd in lst:
            nd.volume = 12345
        huf.setup_nodes(2 * MAXSYM, lst, MAXSYM, fr)
        assert np.array_equal(_nodes(lst), setup)
        assert all(nd.volume == 12345 for nd in lst)   # never touched, as in the reference
        Lc = (C.c_int * (MAXSYM + 1))(*[int(v) for v in L])
        assert huf.find_compressed_data_size(MAXSYM, fr, Lc, 2) == int(size)


@pytest.mark.gpu
def test_generate_and_summarize_tree(gold, huf):
    for f, n, tree, L in zip(gold["tree_freq"], gold["tree_n"], gold["tree_nodes"], gold["tree_lengths"]):
        fr = (C.c_int * (MAXSYM + 1))(*[int(v) for v in f])
        lst = (Node * (2 * MAXSYM))()
        huf.setup_nodes(2 * MAXSYM, lst, MAXSYM, fr)
        huf.generate_huffman_tree(2 * MAXSYM, lst, int(n), MAXSYM)
        got = _nodes(lst)
        bad = np.nonzero((got != tree).any(axis=1))[0]
        assert bad.size == 0, (int(n), bad[:5], got[bad[:3]], tree[bad[:3]])
        out = (C.c_int * (MAXSYM + 1))()
        huf.summarize_tree_with_lengths(2 * MAXSYM, lst, MAXSYM, out, MAXSYM + 1)
        assert np.array_equal(np.array(out[:], np.int32), L)


@pytest.mark.gpu
def test_summarize_reference_test_trees(gold, huf):
    """The two trees of the reference's test_summarize_tree_with_lengths (:1112-1154)."""
    for k, list_length in ((0, 6), (1, 5)):
        rows = gold[f"kat_nodes_{k}"]
        lst = (Node * 6)()
        for i, r in enumerate(rows):
            lst[i] = Node(bool(r[0]), *[int(v) for v in r[1:]], 0)
        out = (C.c_int * (ord("z") + 1))()
        huf.summarize_tree_with_lengths(list_length, lst, ord("z"), out, int(gold[f"kat_leaves_{k}"][0]))
        assert np.array_equal(np.array(out[:], np.int32), gold[f"kat_len_{k}"])
