"""RAPTOR flowchart (.rap) reader and interpreter -- SURVEY.md 8f row f4.

`/root/reference` (Siddarthareddy1/raptor) holds three RAPTOR 4.1 flowcharts
(`RAPTOR/BMI.rap`, `multipication in reverse order.rap`, `summation of digits in 4 digited
number.rap`).  A .rap file is a sequence of .NET
BinaryFormatter streams ([MS-NRBF]): a file version, a few settings, then one stream per
subchart tab (name, kind, the object graph of its flowchart).  This module

* parses MS-NRBF records into plain Python objects (`read_streams`): classes become
  `NObj(cls, members)`, strings `str`, arrays `list`; member references are resolved;
* rebuilds each tab's flowchart (`load`): the start oval's successor chain of components --
  assignment (Rectangle), input / output (Parallelogram), selection (IF_Control with yes /
  no children), loop (Loop: before-test body, exit condition, after-test body), call;
* interprets it (`run`): RAPTOR semantics -- numbers are double precision, identifiers are
  case-insensitive, `+` concatenates when either side is a string, `/` is real division,
  assignments `x <- e` (written `x:=e` in the files), `GET x`, `PUT e`, loops exit when the
  condition is true.

Pure Python, no network, no GPU; it is outside the AMG hot path (SURVEY.md 8f ranks it
last) and exists so a user of the reference finds its one capability here.  Nothing from
the reference is executed or copied: the flowcharts are read as data, like any other input.
"""
from __future__ import annotations

import io
import math
import re
import struct
import sys
from dataclasses import dataclass, field

# ---------------------------------------------------------------------------------------
# MS-NRBF
# ---------------------------------------------------------------------------------------


@dataclass
class NObj:
    cls: str
    members: dict = field(default_factory=dict)

    def get(self, name, default=None):
        return self.members.get(name, default)


class _Ref:
    __slots__ = ("id",)

    def __init__(self, i):
        self.id = i


_PRIM = {1: ("?", 1), 2: ("B", 1), 6: ("d", 8), 7: ("h", 2), 8: ("i", 4), 9: ("q", 8), 10: ("b", 1),
         11: ("f", 4), 12: ("q", 8), 13: ("q", 8), 14: ("H", 2), 15: ("I", 4), 16: ("Q", 8)}


class NrbfReader:
    """One MS-NRBF stream (SerializedStreamHeader ... MessageEnd)."""

    def __init__(self, f: io.BufferedIOBase):
        self.f = f
        self.objs = {}
        self.classes = {}  # object id -> (name, member names, binary types, additional info)
        self.root = None

    # -- primitives --
    def _read(self, n):
        b = self.f.read(n)
        if len(b) != n:
            raise EOFError("truncated MS-NRBF stream")
        return b

    def u8(self):
        return self._read(1)[0]

    def i32(self):
        return struct.unpack("<i", self._read(4))[0]

    def string(self):
        n, shift = 0, 0
        while True:
            b = self.u8()
            n |= (b & 0x7F) << shift
            if not b & 0x80:
                break
            shift += 7
        return self._read(n).decode("utf-8")

    def prim(self, t):
        if t == 18:
            return self.string()
        if t == 5:  # Decimal: as a string
            return float(self.string())
        if t == 3:  # Char: one UTF-8 character
            b = self._read(1)
            need = 0 if b[0] < 0x80 else 1 if b[0] < 0xE0 else 2 if b[0] < 0xF0 else 3
            return (b + self._read(need)).decode("utf-8")
        if t == 17:
            return None
        fmt, n = _PRIM[t]
        return struct.unpack("<" + fmt, self._read(n))[0]

    # -- records --
    def class_info(self):
        oid = self.i32()
        name = self.string()
        cnt = self.i32()
        names = [self.string() for _ in range(cnt)]
        return oid, name, names

    def member_types(self, cnt):
        bts = [self.u8() for _ in range(cnt)]
        extra = []
        for bt in bts:
            if bt in (0, 7):
                extra.append(self.u8())
            elif bt == 3:
                extra.append(self.string())
            elif bt == 4:
                extra.append((self.string(), self.i32()))
            else:
                extra.append(None)
        return bts, extra

    def values(self, oid, name, names, bts, extra):
        members = {}
        for nm, bt, ex in zip(names, bts, extra):
            if bt == 0:
                members[nm] = self.prim(ex)
            else:
                members[nm] = self.record()
        o = NObj(name, members)
        self.objs[oid] = o
        return o

    def record(self):
        rt = self.u8()
        if rt == 0:  # SerializedStreamHeader
            self.root = self.i32()
            self._read(12)
            return self.record()
        if rt == 1:  # ClassWithId
            oid, mid = self.i32(), self.i32()
            name, names, bts, extra = self.classes[mid]
            self.classes[oid] = (name, names, bts, extra)
            return self.values(oid, name, names, bts, extra)
        if rt in (2, 3):  # (System)ClassWithMembers: untyped values
            oid, name, names = self.class_info()
            if rt == 3:
                self.i32()
            bts, extra = [2] * len(names), [None] * len(names)
            self.classes[oid] = (name, names, bts, extra)
            return self.values(oid, name, names, bts, extra)
        if rt in (4, 5):  # (System)ClassWithMembersAndTypes
            oid, name, names = self.class_info()
            bts, extra = self.member_types(len(names))
            if rt == 5:
                self.i32()  # library id
            self.classes[oid] = (name, names, bts, extra)
            return self.values(oid, name, names, bts, extra)
        if rt == 6:  # BinaryObjectString
            oid = self.i32()
            s = self.string()
            self.objs[oid] = s
            return s
        if rt == 7:  # BinaryArray
            oid = self.i32()
            atype = self.u8()
            rank = self.i32()
            lengths = [self.i32() for _ in range(rank)]
            if atype in (3, 4, 5):
                [self.i32() for _ in range(rank)]
            bt = self.u8()
            ex = None
            if bt in (0, 7):
                ex = self.u8()
            elif bt == 3:
                ex = self.string()
            elif bt == 4:
                ex = (self.string(), self.i32())
            n = 1
            for L in lengths:
                n *= L
            out = self._elements(n, prim=ex if bt == 0 else None)
            self.objs[oid] = out
            return out
        if rt == 8:  # MemberPrimitiveTyped
            return self.prim(self.u8())
        if rt == 9:  # MemberReference
            return _Ref(self.i32())
        if rt == 10:
            return None
        if rt == 11:
            return _End
        if rt == 12:  # BinaryLibrary (then the record it precedes)
            self.i32()
            self.string()
            return self.record()
        if rt == 13:
            return _Nulls(self.u8())
        if rt == 14:
            return _Nulls(self.i32())
        if rt == 15:  # ArraySinglePrimitive
            oid, n, t = self.i32(), self.i32(), self.u8()
            out = [self.prim(t) for _ in range(n)]
            self.objs[oid] = out
            return out
        if rt in (16, 17):  # ArraySingleObject / ArraySingleString
            oid, n = self.i32(), self.i32()
            out = self._elements(n)
            self.objs[oid] = out
            return out
        raise ValueError(f"unsupported MS-NRBF record type {rt}")

    def _elements(self, n, prim=None):
        out = []
        while len(out) < n:
            if prim is not None:
                out.append(self.prim(prim))
                continue
            v = self.record()
            if isinstance(v, _Nulls):
                out.extend([None] * v.n)
            else:
                out.append(v)
        return out

    def read(self):
        first = self.record()
        while True:
            r = self.record()
            if r is _End:
                break
        root = self.objs.get(self.root, first)
        return self.resolve(root)

    def resolve(self, v, seen=None):
        seen = set() if seen is None else seen
        if isinstance(v, _Ref):
            v = self.objs[v.id]
        if isinstance(v, NObj):
            if id(v) in seen:
                return v
            seen.add(id(v))
            for k, x in list(v.members.items()):
                v.members[k] = self.resolve(x, seen)
        elif isinstance(v, list):
            for i, x in enumerate(v):
                v[i] = self.resolve(x, seen)
        return v


class _Nulls:
    def __init__(self, n):
        self.n = n


_End = object()


def read_streams(data: bytes):
    """Every MS-NRBF stream of a .rap file, in order, as resolved Python values."""
    f = io.BytesIO(data)
    out = []
    while f.tell() < len(data):
        out.append(NrbfReader(f).read())
    return out


# ---------------------------------------------------------------------------------------
# flowchart model
# ---------------------------------------------------------------------------------------
@dataclass
class Stmt:
    kind: str            # "assign", "input", "output", "if", "loop", "call"
    text: str = ""
    prompt: str = ""
    newline: bool = True
    yes: list = field(default_factory=list)
    no: list = field(default_factory=list)
    before: list = field(default_factory=list)
    after: list = field(default_factory=list)


def _field(o: NObj, *names):
    for n in names:
        for k, v in o.members.items():
            if k == n or k.endswith("+" + n):
                return v
    return None


def _chain(o) -> list:
    """The successor chain starting at component o (ovals contribute nothing)."""
    out = []
    while isinstance(o, NObj):
        st = _stmt(o)
        if st is not None:
            out.append(st)
        o = _field(o, "_Successor", "Successor")
    return out


def _text(o):
    t = _field(o, "_text_str", "text_str")
    return t if isinstance(t, str) else ""


def _stmt(o: NObj):
    cls = o.cls.split(".")[-1]
    if cls == "Oval":
        return None
    if cls == "Rectangle":
        kind = _field(o, "_kind", "kind")
        kind = kind.get("value__", 0) if isinstance(kind, NObj) else (kind or 0)
        return Stmt("call" if kind == 1 else "assign", text=_text(o))
    if cls == "Parallelogram":
        is_input = bool(_field(o, "_is_input", "is_input"))
        prompt = _field(o, "_prompt", "prompt") or ""
        nl = _field(o, "_new_line", "new_line")
        return Stmt("input" if is_input else "output", text=_text(o), prompt=prompt,
                    newline=True if nl is None else bool(nl))
    if cls == "IF_Control":  # RAPTOR draws the yes branch on the left
        return Stmt("if", text=_text(o), yes=_chain(_field(o, "_left_Child", "yes_child")),
                    no=_chain(_field(o, "_right_Child", "no_child")))
    if cls == "Loop":
        return Stmt("loop", text=_text(o), before=_chain(_field(o, "_before_Child", "before_Child")),
                    after=_chain(_field(o, "_after_Child", "after_Child")))
    raise ValueError(f"unknown RAPTOR component {o.cls}")


@dataclass
class Flowchart:
    version: object
    tabs: dict  # tab name -> list[Stmt]


def load(path_or_bytes) -> Flowchart:
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    streams = read_streams(bytes(data))
    version = streams[0]
    tabs = {}
    i = 1
    while i < len(streams):
        v = streams[i]
        # a tab: its name, then (4.x) its kind, then the start oval
        if isinstance(v, str) and i + 1 < len(streams):
            j = i + 1
            while j < len(streams) and not (isinstance(streams[j], NObj) and streams[j].cls.endswith("Oval")):
                j += 1
            if j < len(streams):
                tabs[v] = _chain(streams[j])
                i = j + 1
                continue
        i += 1
    return Flowchart(version, tabs)


# ---------------------------------------------------------------------------------------
# expressions and execution
# ---------------------------------------------------------------------------------------
_TOK = re.compile(r'\s*(?:(?P<num>\d+\.?\d*(?:[eE][-+]?\d+)?|\.\d+)|(?P<str>"[^"]*")|'
                  r'(?P<id>[A-Za-z_][A-Za-z_0-9]*)|(?P<op>&&|\|\||<=|>=|!=|/=|==|<-|:=|\*\*|[-+*/^<>=(),\[\]!]))')


def _tokens(s):
    pos, out = 0, []
    s = s.strip()
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            raise SyntaxError(f"bad expression near {s[pos:]!r}")
        pos = m.end()
        for k in ("num", "str", "id", "op"):
            if m.group(k) is not None:
                out.append((k, m.group(k)))
                break
    return out


_FUNCS = {"sqrt": math.sqrt, "abs": abs, "floor": math.floor, "ceiling": math.ceil, "sin": math.sin,
          "cos": math.cos, "tan": math.tan, "log": math.log, "exp": math.exp, "min": min, "max": max,
          "arctan": math.atan, "arcsin": math.asin, "arccos": math.acos}
_CONST = {"pi": math.pi, "e": math.e, "true": True, "false": False}


class _Parser:
    """RAPTOR expressions: or / and / not, comparisons, + - (left assoc), * / mod rem,
    ^ / ** (right assoc), unary minus, numbers, strings, variables, calls."""

    def __init__(self, toks, env):
        self.t, self.i, self.env = toks, 0, env

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else (None, None)

    def take(self, v=None):
        k, x = self.peek()
        if v is not None and (x is None or x.lower() != v):
            raise SyntaxError(f"expected {v!r}, got {x!r}")
        self.i += 1
        return k, x

    def parse(self):
        v = self.or_()
        if self.i != len(self.t):
            raise SyntaxError(f"trailing tokens {self.t[self.i:]}")
        return v

    def or_(self):
        v = self.and_()
        while (self.peek()[1] or "").lower() in ("or", "||"):
            self.take()
            r = self.and_()
            v = bool(v) or bool(r)
        return v

    def and_(self):
        v = self.not_()
        while (self.peek()[1] or "").lower() in ("and", "&&"):
            self.take()
            r = self.not_()
            v = bool(v) and bool(r)
        return v

    def not_(self):
        if (self.peek()[1] or "").lower() in ("not", "!"):
            self.take()
            return not self.not_()
        return self.cmp()

    def cmp(self):
        v = self.add()
        op = self.peek()[1]
        if op in ("<", ">", "<=", ">=", "=", "==", "!=", "/="):
            self.take()
            r = self.add()
            return {"<": v < r, ">": v > r, "<=": v <= r, ">=": v >= r, "=": v == r, "==": v == r,
                    "!=": v != r, "/=": v != r}[op]
        return v

    def add(self):
        v = self.mul()
        while self.peek()[1] in ("+", "-"):
            op = self.take()[1]
            r = self.mul()
            if op == "+" and (isinstance(v, str) or isinstance(r, str)):
                v = _show(v) + _show(r)
            else:
                v = v + r if op == "+" else v - r
        return v

    def mul(self):
        v = self.pow_()
        while self.peek()[1] in ("*", "/") or (self.peek()[1] or "").lower() in ("mod", "rem"):
            op = self.take()[1].lower()
            r = self.pow_()
            if op == "*":
                v = v * r
            elif op == "/":
                v = v / r
            elif op == "mod":
                v = v - r * math.floor(v / r)
            else:
                v = math.fmod(v, r)
        return v

    def pow_(self):
        v = self.unary()
        if self.peek()[1] in ("^", "**"):
            self.take()
            return v ** self.pow_()
        return v

    def unary(self):
        if self.peek()[1] == "-":
            self.take()
            return -self.unary()
        if self.peek()[1] == "+":
            self.take()
            return self.unary()
        return self.atom()

    def atom(self):
        k, x = self.take()
        if k == "num":
            return float(x)
        if k == "str":
            return x[1:-1]
        if x == "(":
            v = self.or_()
            self.take(")")
            return v
        if k == "id":
            name = x.lower()
            if self.peek()[1] == "(":
                self.take()
                args = [self.or_()]
                while self.peek()[1] == ",":
                    self.take()
                    args.append(self.or_())
                self.take(")")
                if name not in _FUNCS:
                    raise NameError(f"unknown function {x}")
                return float(_FUNCS[name](*args))
            if name in self.env:
                return self.env[name]
            if name in _CONST:
                return _CONST[name]
            raise NameError(f"variable {x} has no value")
        raise SyntaxError(f"unexpected {x!r}")


def evaluate(expr: str, env: dict):
    return _Parser(_tokens(expr), env).parse()


def _show(v):
    """RAPTOR prints whole numbers without a decimal point."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        if math.isfinite(v) and v == int(v):
            return str(int(v))
        r = f"{v:.4f}".rstrip("0").rstrip(".")
        return r
    return str(v)


class Machine:
    def __init__(self, inputs=(), max_steps=1_000_000):
        self.inputs = list(inputs)
        self.out = []          # completed output lines
        self.line = ""
        self.env = {}
        self.steps = 0
        self.max_steps = max_steps
        self.prompts = []       # the prompt expression of every GET, in order

    def _get(self, prompt):
        self.prompts.append(prompt)
        if not self.inputs:
            raise EOFError(f"no input left for {prompt!r}")
        v = self.inputs.pop(0)
        if isinstance(v, str):
            try:
                return float(v)
            except ValueError:
                return v
        return float(v)

    def exec(self, body):
        for st in body:
            self.steps += 1
            if self.steps > self.max_steps:
                raise RuntimeError("step limit reached")
            if st.kind == "assign":
                lhs, rhs = re.split(r"\s*(?::=|<-|←)\s*", st.text.strip(), maxsplit=1)
                self.env[lhs.strip().lower()] = evaluate(rhs, self.env)
            elif st.kind == "input":
                self.env[st.text.strip().lower()] = self._get(st.prompt)
            elif st.kind == "output":
                self.line += _show(evaluate(st.text, self.env))
                if st.newline:
                    self.out.append(self.line)
                    self.line = ""
            elif st.kind == "if":
                self.exec(st.yes if evaluate(st.text, self.env) else st.no)
            elif st.kind == "loop":
                while True:
                    self.exec(st.before)
                    if evaluate(st.text, self.env):
                        break
                    self.exec(st.after)
            elif st.kind == "call":
                raise NotImplementedError(f"subchart / procedure call {st.text!r}")
        return self


def run(chart: Flowchart, inputs=(), tab="main"):
    """Run tab `tab` with the given inputs; returns the output lines."""
    m = Machine(inputs)
    m.exec(chart.tabs[tab])
    if m.line:
        m.out.append(m.line)
    return m.out


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="Run a RAPTOR .rap flowchart")
    ap.add_argument("path")
    ap.add_argument("inputs", nargs="*", help="values for the flowchart's GET statements, in order")
    ap.add_argument("--dump", action="store_true", help="print the flowchart instead of running it")
    a = ap.parse_args(argv)
    fc = load(a.path)
    if a.dump:
        for name, body in fc.tabs.items():
            print(f"tab {name}:")
            _dump(body, 1)
        return 0
    for line in run(fc, a.inputs):
        print(line)
    return 0


def _dump(body, depth):
    pad = "  " * depth
    for st in body:
        if st.kind == "if":
            print(f"{pad}IF {st.text}")
            _dump(st.yes, depth + 1)
            print(f"{pad}ELSE")
            _dump(st.no, depth + 1)
        elif st.kind == "loop":
            print(f"{pad}LOOP")
            _dump(st.before, depth + 1)
            print(f"{pad}EXIT WHEN {st.text}")
            _dump(st.after, depth + 1)
        else:
            print(f"{pad}{st.kind.upper()} {st.prompt + ' -> ' if st.prompt else ''}{st.text}")


if __name__ == "__main__":
    sys.exit(main())
