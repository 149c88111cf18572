"""A pickle *reader* that never executes anything.

The reference persists its training flags as a Python-2 pickle of an
``argparse.Namespace`` (``train.py:54-55``; ``save/kanji/config.pkl``).
Unpickling runs arbitrary callables, so instead this module interprets the
pickle opcode stream (protocols 0-2) as pure data: ``GLOBAL`` references are
recorded as names and never imported, ``REDUCE``/``NEWOBJ``/``BUILD`` only
produce :class:`Reconstructed` records holding the state they would have
set. Anything outside the supported opcode subset raises ``ValueError``.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List


@dataclass
class Global:
    module: str
    name: str

    @property
    def qualname(self) -> str:
        return self.module + "." + self.name


@dataclass
class Reconstructed:
    callable: Any
    args: Any
    state: Dict[str, Any] = field(default_factory=dict)


class _Mark:
    pass


_MARK = _Mark()


def _decode_py2_string(s: str) -> str:
    # protocol-0 STRING is a repr() of a byte string
    body = s.strip()
    if len(body) >= 2 and body[0] == body[-1] and body[0] in "'\"":
        body = body[1:-1]
    return body.encode("latin1").decode("unicode_escape")


def loads(data: bytes) -> Any:
    stack: List[Any] = []
    memo: Dict[int, Any] = {}
    pos = 0
    n = len(data)

    def readline() -> str:
        nonlocal pos
        end = data.index(b"\n", pos)
        line = data[pos:end].decode("latin1")
        pos = end + 1
        return line

    def read(k: int) -> bytes:
        nonlocal pos
        if pos + k > n:
            raise ValueError("truncated pickle")
        b = data[pos:pos + k]
        pos += k
        return b

    def pop_mark() -> List[Any]:
        items = []
        while True:
            x = stack.pop()
            if x is _MARK:
                break
            items.append(x)
        items.reverse()
        return items

    while pos < n:
        op = data[pos:pos + 1]
        pos += 1
        if op == b"\x80":  # PROTO
            read(1)
        elif op == b".":  # STOP
            return stack.pop()
        elif op == b"(":
            stack.append(_MARK)
        elif op == b"c":  # GLOBAL
            mod = readline()
            name = readline()
            stack.append(Global(mod, name))
        elif op == b"N":
            stack.append(None)
        elif op == b"\x88":
            stack.append(True)
        elif op == b"\x89":
            stack.append(False)
        elif op == b"I":
            line = readline()
            stack.append(True if line == "01" else False if line == "00" else int(line))
        elif op == b"L":
            stack.append(int(readline().rstrip("L")))
        elif op == b"F":
            stack.append(float(readline()))
        elif op == b"G":
            stack.append(struct.unpack(">d", read(8))[0])
        elif op == b"J":
            stack.append(struct.unpack("<i", read(4))[0])
        elif op == b"K":
            stack.append(read(1)[0])
        elif op == b"M":
            stack.append(struct.unpack("<H", read(2))[0])
        elif op == b"S":
            stack.append(_decode_py2_string(readline()))
        elif op == b"V":
            stack.append(readline().encode("latin1").decode("raw_unicode_escape"))
        elif op == b"U":
            k = read(1)[0]
            stack.append(read(k).decode("latin1"))
        elif op == b"T":
            k = struct.unpack("<I", read(4))[0]
            stack.append(read(k).decode("latin1"))
        elif op == b"X":
            k = struct.unpack("<I", read(4))[0]
            stack.append(read(k).decode("utf-8"))
        elif op == b"p":
            memo[int(readline())] = stack[-1]
        elif op == b"q":
            memo[read(1)[0]] = stack[-1]
        elif op == b"r":
            memo[struct.unpack("<I", read(4))[0]] = stack[-1]
        elif op == b"g":
            stack.append(memo[int(readline())])
        elif op == b"h":
            stack.append(memo[read(1)[0]])
        elif op == b"j":
            stack.append(memo[struct.unpack("<I", read(4))[0]])
        elif op == b"t":
            stack.append(tuple(pop_mark()))
        elif op == b")":
            stack.append(())
        elif op == b"\x85":
            stack.append((stack.pop(),))
        elif op == b"\x86":
            b_ = stack.pop()
            a_ = stack.pop()
            stack.append((a_, b_))
        elif op == b"\x87":
            c_ = stack.pop()
            b_ = stack.pop()
            a_ = stack.pop()
            stack.append((a_, b_, c_))
        elif op == b"l":
            stack.append(pop_mark())
        elif op == b"]":
            stack.append([])
        elif op == b"a":
            v = stack.pop()
            stack[-1].append(v)
        elif op == b"e":
            items = pop_mark()
            stack[-1].extend(items)
        elif op == b"d":
            items = pop_mark()
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif op == b"}":
            stack.append({})
        elif op == b"s":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif op == b"u":
            items = pop_mark()
            for i in range(0, len(items), 2):
                stack[-1][items[i]] = items[i + 1]
        elif op == b"R":  # REDUCE: record, never call
            args = stack.pop()
            fn = stack.pop()
            stack.append(Reconstructed(fn, args))
        elif op == b"\x81":  # NEWOBJ
            args = stack.pop()
            cls = stack.pop()
            stack.append(Reconstructed(cls, args))
        elif op == b"b":  # BUILD
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, Reconstructed) and isinstance(state, dict):
                obj.state.update(state)
            else:
                raise ValueError("BUILD on unsupported object")
        elif op == b"0":
            stack.pop()
        elif op == b"2":
            stack.append(stack[-1])
        else:
            raise ValueError("unsupported pickle opcode %r at %d" % (op, pos - 1))
    raise ValueError("pickle without STOP")


def load_namespace_pickle(path: str) -> Dict[str, Any]:
    """Return the attribute dict of a pickled ``argparse.Namespace``."""
    with open(path, "rb") as f:
        obj = loads(f.read())
    if isinstance(obj, Reconstructed):
        # copy_reg._reconstructor(cls, base, state) + BUILD dict
        cls = obj.args[0] if isinstance(obj.args, tuple) and obj.args else obj.callable
        if isinstance(cls, Global) and cls.name != "Namespace":
            raise ValueError("expected an argparse.Namespace, found %s" % cls.qualname)
        return dict(obj.state)
    if isinstance(obj, dict):
        return obj
    raise ValueError("unexpected pickle payload %r" % type(obj))
