"""RAPTOR .rap reader / interpreter (raptor_amd/rap.py).  CPU only.

Two kinds of checks:
* synthetic MS-NRBF streams written by the small encoder below (records the reader must
  handle: class with members and types, class with id, strings, member references, nulls,
  primitives) and flowcharts built from them -- independent of the reference;
* the reference's own three flowcharts, read from /root/reference as data when it is present
  (this container; never on the GPU box), against the semantics SURVEY.md Appendix A records:
  BMI prints w/h*h = w and classifies with strict inequalities (18.5, 25 and 30 fall through to
  "Overweight"); the reverse multiplication loop prints 10n .. 0 then "n mul is over"; the
  digit sum prints a+b+c+d."""
import io
import os
import struct

import pytest

from raptor_amd import rap as R

REF = "/root/reference/RAPTOR"


# ---- a minimal MS-NRBF encoder (test helper) --------------------------------------------
def _s(x):
    b = x.encode()
    n, out = len(b), bytearray()
    while True:
        c = n & 0x7F
        n >>= 7
        out.append(c | (0x80 if n else 0))
        if not n:
            break
    return bytes(out) + b


class Enc:
    """Writes NObj graphs: primitive members typed (Int32 / Boolean / Double / String
    members as BinaryObjectString), object members as records or references."""

    def __init__(self):
        self.buf = io.BytesIO()
        self.next_id = 1
        self.ids = {}
        self.classes = {}

    def _id(self):
        i = self.next_id
        self.next_id += 1
        return i

    def obj(self, o):
        if o is None:
            self.buf.write(b"\x0a")
            return
        if isinstance(o, str):
            self.buf.write(b"\x06" + struct.pack("<i", self._id()) + _s(o))
            return
        if id(o) in self.ids:
            self.buf.write(b"\x09" + struct.pack("<i", self.ids[id(o)]))
            return
        oid = self._id()
        self.ids[id(o)] = oid
        names = list(o.members)
        if o.cls in self.classes:  # ClassWithId
            self.buf.write(b"\x01" + struct.pack("<ii", oid, self.classes[o.cls]))
        else:
            self.classes[o.cls] = oid
            self.buf.write(b"\x05" + struct.pack("<i", oid) + _s(o.cls) + struct.pack("<i", len(names)))
            for nm in names:
                self.buf.write(_s(nm))
            types = [self._btype(o.members[nm]) for nm in names]
            self.buf.write(bytes(t for t, _ in types))
            for t, ex in types:
                if ex is not None:
                    self.buf.write(bytes([ex]))
            self.buf.write(struct.pack("<i", 2))  # library id
        for nm in names:
            v = o.members[nm]
            t, ex = self._btype(v)
            if t == 0:
                self.buf.write(struct.pack({1: "<?", 8: "<i", 6: "<d"}[ex], v))
            else:
                self.obj(v)

    @staticmethod
    def _btype(v):
        if isinstance(v, bool):
            return 0, 1
        if isinstance(v, int):
            return 0, 8
        if isinstance(v, float):
            return 0, 6
        if isinstance(v, str):
            return 1, None
        return 2, None

    def stream(self, root):
        self.buf.write(b"\x00" + struct.pack("<iiii", 1, -1, 1, 0))
        self.buf.write(b"\x0c" + struct.pack("<i", 2) + _s("raptor, Version=4.1.0.1"))
        self.obj(root)
        self.buf.write(b"\x0b")
        self.ids, self.classes, self.next_id = {}, {}, 1
        return self


def comp(cls, text="", succ=None, **kw):
    m = {"_serialization_version": 17, "_text_str": text, "_Successor": succ}
    m.update(kw)
    return R.NObj("raptor." + cls, m)


def encode(start):
    e = Enc()
    e.stream(R.NObj("System.Int32", {"m_value": 17}))
    e.stream("main")
    e.stream(R.NObj("raptor.Subchart_Kinds", {"value__": 0}))
    e.stream(start)
    return e.buf.getvalue()


def link(*cs, end=None):
    for a, b in zip(cs, cs[1:]):
        a.members["_Successor"] = b
    cs[-1].members["_Successor"] = end
    return cs[0]


def par(text, is_input, prompt=""):
    return comp("Parallelogram", text, _prompt=prompt, _is_input=is_input, _new_line=True)


def rect(text):
    return comp("Rectangle", text, _kind=R.NObj("raptor.Rectangle+Kind_Of", {"value__": 0}))


# ---- synthetic -------------------------------------------------------------------------
def test_nrbf_records_roundtrip():
    shared = R.NObj("X.Shared", {"v": 3.5})
    root = R.NObj("X.Root", {"a": 7, "b": True, "s": "hello", "p": shared, "q": shared, "n": None})
    e = Enc().stream(root)
    (got,) = R.read_streams(e.buf.getvalue())
    assert got.cls == "X.Root" and got.get("a") == 7 and got.get("b") is True
    assert got.get("s") == "hello" and got.get("n") is None
    assert got.get("p") is got.get("q") and got.get("p").get("v") == 3.5  # reference resolved


def test_interpreter_semantics():
    end = comp("Oval", "End")
    # GET x ; y := 2^3 + x mod 4 ; IF y > 10 && !(x = 0) THEN PUT "big " + y ELSE PUT y
    # LOOP: k := k + 1 ; EXIT WHEN k >= 3 ; PUT k
    yes = link(par('"big " + y', False))
    no = link(par("y", False))
    ifc = comp("IF_Control", "y > 10 && !(x = 0)", _left_Child=yes, _right_Child=no)
    loop = comp("Loop", "k >= 3", _before_Child=link(rect("k:=k+1")), _after_Child=link(par("k", False)))
    body = link(par("x", True, '"x?"'), rect("y:=2^3+x mod 4"), ifc, rect("K:=0"), loop, end=end)
    start = comp("Oval", "Start", succ=body)
    fc = R.load(encode(start))
    assert list(fc.tabs) == ["main"]
    assert R.run(fc, [7]) == ["big 11", "1", "2"]
    assert R.run(fc, [1]) == ["9", "1", "2"]          # 8 + 1 mod 4 = 9, not > 10
    assert R.evaluate("7 / 2 * 2", {}) == 7.0           # left associative, real division
    assert R.evaluate("2 ^ 3 ^ 2", {}) == 512.0          # right associative
    assert R.evaluate("-7 mod 3", {}) == 2.0 and R.evaluate("-7 rem 3", {}) == -1.0
    with pytest.raises(NameError):
        R.evaluate("undefined + 1", {})


# ---- the reference's flowcharts (data files read in place) --------------------------------
need_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")


# The first output line is BMI:=w/h*h = (w/h)*h, i.e. the weight.  The expected strings are
# literals; how RAPTOR itself prints non-integer numbers (here: shortest form, no trailing
# zeros) is not pinned by anything the reference holds -- parity of the number format is
# unpinned, only the values and the branch taken are.
@need_ref
@pytest.mark.parametrize("h,w,shown,cls", [(1.8, 70, "70", "Overweight"), (1, 18.5, "18.5", "Overweight"),
                                           (1, 20, "20", "Healthy weight"), (1, 25, "25", "Overweight"),
                                           (1, 27.5, "27.5", "At risk of overweight"),
                                           (1, 30, "30", "Overweight"), (2, 10, "10", "UnderWeight")])
def test_reference_bmi(h, w, shown, cls):
    fc = R.load(os.path.join(REF, "BMI.rap"))
    out = R.run(fc, [h, w])
    assert out == [shown, cls]


@need_ref
@pytest.mark.parametrize("n", [7, 3, 0])
def test_reference_reverse_multiplication(n):
    fc = R.load(os.path.join(REF, "multipication in reverse order.rap"))
    assert R.run(fc, [n]) == [str(n * i) for i in range(10, -1, -1)] + [f"{n} mul is over"]


@need_ref
@pytest.mark.parametrize("digits", [(1, 2, 3, 4), (9, 9, 9, 9), (12, 0, 5, 1)])
def test_reference_digit_sum(digits):
    fc = R.load(os.path.join(REF, "summation of digits in 4 digited number.rap"))
    assert R.run(fc, list(digits)) == [str(sum(digits))]
