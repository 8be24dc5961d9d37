#!/usr/bin/env python3
"""Config C1 fixture: the message /root/reference/c++/samples/addressbook.c++:47-76 writes.

The sample needs generated code (capnpc-c++ output for samples/addressbook.capnp), which is not
built here.  Its message is small enough to lay out by hand instead: MallocMessageBuilder places
objects in one segment in the order the sample initialises them (root struct, the people list,
then each text / list as it is set), with the struct layouts the schema compiler assigns to
samples/addressbook.capnp:

    Person       1 data word (id: UInt32 @ bits 0-31, employment discriminant: UInt16 @ 32-47),
                 4 pointers (name, email, phones, employer|school)
    PhoneNumber  1 data word (type: UInt16 @ bits 0-15), 1 pointer (number)
    AddressBook  0 data words, 1 pointer (people)

The result is pinned to the reference itself by SURVEY.md 8(c), which recorded the sha256 of the
288-byte message and of its 151-byte packed form as produced by the compiled sample
(6734639c...9b7b and 6cb6a027...39189).  The packed form is produced here by the reference codec
(oracle/_ref) and checked against that hash too.  Writes tests/golden/addressbook.bin (flat:
segment table + segment) and tests/golden/addressbook.packed.
"""
import hashlib
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle")]

MSG_SHA = ("6734639c", "9b7b")
PACKED_SHA = ("6cb6a027", "39189")


def struct_ptr(offset, data, ptrs):
    return ((offset << 2) & 0xFFFFFFFF) | (data << 32) | (ptrs << 48)


def list_ptr(offset, elem_size, count):
    return 1 | ((offset << 2) & 0xFFFFFFFF) | (elem_size << 32) | (count << 35)


def build():
    seg = [0] * 64
    top = [0]

    def alloc(n):
        a = top[0]
        top[0] += n
        return a

    def text(ptr_at, s):
        b = s.encode() + b"\0"
        n = (len(b) + 7) // 8
        at = alloc(n)
        raw = b + b"\0" * (8 * n - len(b))
        for i in range(n):
            seg[at + i] = struct.unpack_from("<Q", raw, 8 * i)[0]
        seg[ptr_at] = list_ptr(at - (ptr_at + 1), 2, len(b))

    def struct_list(ptr_at, count, data, ptrs):
        at = alloc(1 + count * (data + ptrs))
        seg[at] = struct_ptr(count, data, ptrs)  # tag word: element count in the offset field
        seg[ptr_at] = list_ptr(at - (ptr_at + 1), 7, count * (data + ptrs))
        return [at + 1 + i * (data + ptrs) for i in range(count)]

    root = alloc(1)
    book = alloc(1)  # AddressBook: 0 data words, 1 pointer
    seg[root] = struct_ptr(book - (root + 1), 0, 1)
    alice, bob = struct_list(book, 2, 1, 4)  # initPeople(2)

    def person(p, pid, name, email, phones, school):
        seg[p] |= pid
        text(p + 1, name)
        text(p + 2, email)
        els = struct_list(p + 3, len(phones), 1, 1)
        for e, (num, typ) in zip(els, phones):
            text(e + 1, num)
            seg[e] |= typ
        if school is not None:  # employment.setSchool: discriminant 2, then the text
            seg[p] |= 2 << 32
            text(p + 4, school)
        # setUnemployed: discriminant 0 (already zero)

    person(alice, 123, "Alice", "alice@example.com", [("555-1212", 0)], "MIT")
    person(bob, 456, "Bob", "bob@example.com", [("555-4567", 1), ("555-7654", 2)], None)
    n = top[0]
    table = struct.pack("<II", 0, n)
    return table + b"".join(struct.pack("<Q", w) for w in seg[:n])


def check(b, pin, what):
    h = hashlib.sha256(b).hexdigest()
    if not (h.startswith(pin[0]) and h.endswith(pin[1])):
        raise SystemExit(f"{what}: sha256 {h} does not match the reference's {pin[0]}...{pin[1]}")
    return h


def main():
    import numpy as np
    import pyoracle as P

    msg = build()
    assert len(msg) == 288, len(msg)
    check(msg, MSG_SHA, "message")
    words = np.frombuffer(msg, "<u8")
    packed = P.Reference().pack_segments(P.split_flat(words))
    assert len(packed) == 151, len(packed)
    h = check(packed, PACKED_SHA, "packed")
    g = os.path.join(ROOT, "tests", "golden")
    open(os.path.join(g, "addressbook.bin"), "wb").write(msg)
    open(os.path.join(g, "addressbook.packed"), "wb").write(packed)
    print("addressbook: 288 B -> 151 B, sha256", hashlib.sha256(msg).hexdigest(), h)


if __name__ == "__main__":
    main()
