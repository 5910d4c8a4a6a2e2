"""oracle.check_utf8 (arrow2 0.17 try_check_utf8, the check behind
Utf8Array::try_new at read/array/binary.rs:305-306) on hand cases, and its
UTF-8 acceptor pinned against the Unicode Standard's table of well-formed
byte sequences (Table 3-7), which is what simdutf8 validates."""
import numpy as np

from oracle import oracle as O

# Unicode 15 Table 3-7: (first byte range, then the ranges of the trail bytes)
TABLE_3_7 = [
    ((0x00, 0x7F),),
    ((0xC2, 0xDF), (0x80, 0xBF)),
    ((0xE0, 0xE0), (0xA0, 0xBF), (0x80, 0xBF)),
    ((0xE1, 0xEC), (0x80, 0xBF), (0x80, 0xBF)),
    ((0xED, 0xED), (0x80, 0x9F), (0x80, 0xBF)),
    ((0xEE, 0xEF), (0x80, 0xBF), (0x80, 0xBF)),
    ((0xF0, 0xF0), (0x90, 0xBF), (0x80, 0xBF), (0x80, 0xBF)),
    ((0xF1, 0xF3), (0x80, 0xBF), (0x80, 0xBF), (0x80, 0xBF)),
    ((0xF4, 0xF4), (0x80, 0x8F), (0x80, 0xBF), (0x80, 0xBF)),
]


def well_formed(b: bytes) -> bool:
    i = 0
    while i < len(b):
        for row in TABLE_3_7:
            if i + len(row) <= len(b) and all(lo <= b[i + k] <= hi for k, (lo, hi) in enumerate(row)):
                i += len(row)
                break
        else:
            return False
    return True


def test_acceptor_matches_table_3_7():
    rng = np.random.default_rng(0)
    interesting = [0x00, 0x41, 0x7F, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC,
                   0xED, 0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xFF]
    for a in interesting:  # every 1- and 2-byte sequence of boundary bytes, then random 3-6 byte ones
        for b in interesting:
            for s in (bytes([a]), bytes([a, b])):
                assert O.check_utf8(s, [0, len(s)]) == well_formed(s), s
    for _ in range(20000):
        s = bytes(rng.choice(interesting, int(rng.integers(1, 7))))
        assert O.check_utf8(s, [0, len(s)]) == well_formed(s), s


def test_offsets_rule():
    e = "é".encode()  # c3 a9
    assert O.check_utf8(b"", [0])
    assert O.check_utf8(e, [0])  # no rows: nothing checked
    assert O.check_utf8(e, [0, 2])
    assert not O.check_utf8(e, [0, 1, 2])  # offset 1 inside the character
    assert O.check_utf8(e, [1, 2])  # offset 0 is checked only up to `last` (none here)
    assert not O.check_utf8(e, [1, 1, 2])
    assert O.check_utf8(b"ab\xc3\xa9", [0, 1, 4])
    assert O.check_utf8(b"ab\xff", [0, 2]) is False  # the whole buffer is checked, past the last offset too
    assert O.check_utf8(b"abc", [0, 1, 2, 3])  # ASCII: no boundary check
