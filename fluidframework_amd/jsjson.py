"""JS-compatible JSON text for interned property keys/values.

The engine never parses JSON: the host interns every property key and value of
an op once, and the snapshot writer splices their pre-serialized text.  The text
must be byte-identical to V8's ``JSON.stringify`` (Node >= 12, well-formed
stringify), which is what the reference's serializer produces
(``packages/runtime/runtime-utils/src/serializer.ts:42-54`` -> JSON.stringify).

Rules restated here:
* strings are sequences of UTF-16 code units; ``"``/``\\``/``\\b\\f\\n\\r\\t`` use
  short escapes, other C0 controls ``\\u00xx`` (lowercase), lone surrogates
  ``\\udxxx`` (lowercase), everything else is emitted as UTF-8;
* numbers follow ECMAScript Number::toString; NaN/Infinity serialize as null;
* object members enumerate array-index keys ascending first, then the other
  keys in insertion order (OrdinaryOwnPropertyKeys).
"""
from __future__ import annotations

import math
import re
from typing import Any

class _Undefined:
    """JS `undefined` as a property value (a key that is present with value undefined, e.g. what a
    combining op with an unknown name and no defaultValue stores): JSON.stringify skips such
    object members and writes null for such array elements."""
    __slots__ = ()

    def __repr__(self):
        return "undefined"


UNDEFINED = _Undefined()

_SHORT = {0x22: '\\"', 0x5C: "\\\\", 0x08: "\\b", 0x0C: "\\f", 0x0A: "\\n", 0x0D: "\\r", 0x09: "\\t"}


def utf16_units(s: str) -> list[int]:
    """UTF-16 code units of a Python str (lone surrogates kept as-is)."""
    b = s.encode("utf-16-le", "surrogatepass")
    return [b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2)]


def quote_units(units) -> str:
    out = ['"']
    n = len(units)
    i = 0
    while i < n:
        c = units[i]
        if c in _SHORT:
            out.append(_SHORT[c])
        elif c < 0x20:
            out.append("\\u%04x" % c)
        elif 0xD800 <= c <= 0xDBFF and i + 1 < n and 0xDC00 <= units[i + 1] <= 0xDFFF:
            cp = 0x10000 + ((c - 0xD800) << 10) + (units[i + 1] - 0xDC00)
            out.append(chr(cp))
            i += 1
        elif 0xD800 <= c <= 0xDFFF:
            out.append("\\u%04x" % c)
        else:
            out.append(chr(c))
        i += 1
    out.append('"')
    return "".join(out)


def quote(s: str) -> str:
    return quote_units(utf16_units(s))


def number_to_js(v: float) -> str:
    if isinstance(v, bool):
        raise TypeError("bool is not a number")
    if isinstance(v, int):
        if abs(v) < 10**21:
            return str(v)
        v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "-Infinity" if v < 0 else "Infinity"
    if v == 0:
        return "0"
    sign = "-" if v < 0 else ""
    v = abs(v)
    r = repr(v)  # shortest round-trip digits
    mant, _, exp = r.partition("e")
    ex = int(exp) if exp else 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    n = len(ip) + ex - lead_zeros  # decimal point position relative to digits
    digits = digits.rstrip("0") or "0"
    k = len(digits)
    if k <= n <= 21:
        s = digits + "0" * (n - k)
    elif 0 < n <= 21:
        s = digits[:n] + "." + digits[n:]
    elif -6 < n <= 0:
        s = "0." + "0" * (-n) + digits
    else:
        e1 = n - 1
        s = digits[0] + ("." + digits[1:] if k > 1 else "") + "e" + ("-" if e1 < 0 else "+") + str(abs(e1))
    return sign + s


def array_index(key: str):
    if not key or len(key) > 10 or not key.isdigit() or not key.isascii():
        return None
    if len(key) > 1 and key[0] == "0":
        return None
    v = int(key)
    return v if v < 4294967295 else None


def js_key_order(keys) -> list:
    idx = sorted((array_index(k), k) for k in keys if array_index(k) is not None)
    rest = [k for k in keys if array_index(k) is None]
    return [k for _, k in idx] + rest


def stringify(v: Any) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, (int, float)):
        if isinstance(v, float) and not math.isfinite(v):
            return "null"
        return number_to_js(v)
    if isinstance(v, str):
        return quote(v)
    if isinstance(v, (list, tuple)):
        return "[" + ",".join("null" if x is UNDEFINED else stringify(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ",".join(quote(k) + ":" + stringify(v[k]) for k in js_key_order(list(v.keys()))
                              if v[k] is not UNDEFINED) + "}"
    raise TypeError(f"not a JSON value: {type(v)}")


def js_truthy(v: Any) -> bool:
    if v is None or v is False or v is UNDEFINED:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return not (v == 0 or (isinstance(v, float) and math.isnan(v)))
    if isinstance(v, str):
        return len(v) > 0
    return True


def match_class_key(v: Any):
    """Canonical form under MT/properties.ts:64-95 matchProperties equality.

    Objects compare order-insensitively and recursively; arrays behave as
    objects keyed by index; primitives compare with ``===``.  (Mixed
    primitive/object comparisons are not canonicalized; see DESIGN.md.)
    """
    if isinstance(v, dict):
        return ("o", tuple(sorted((k, match_class_key(x)) for k, x in v.items())))
    if isinstance(v, (list, tuple)):
        return ("o", tuple(sorted((str(i), match_class_key(x)) for i, x in enumerate(v))))
    if isinstance(v, bool):
        return ("b", v)
    if isinstance(v, (int, float)):
        return ("n", float(v))
    if isinstance(v, str):
        return ("s", v)
    return ("z", None)


# StrWhiteSpaceChar (ECMA-262 7.1.4.1.1): WhiteSpace and LineTerminator
_JS_WS = "\t\n\v\f\r \u00a0\u1680\u2000\u2001\u2002\u2003\u2004\u2005\u2006\u2007\u2008\u2009\u200a" \
         "\u2028\u2029\u202f\u205f\u3000\ufeff"
_JS_DEC = re.compile(r"[+-]?(?:(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?|Infinity)\Z")
_JS_RADIX = {"0x": (16, re.compile(r"[0-9a-fA-F]+\Z")), "0o": (8, re.compile(r"[0-7]+\Z")),
             "0b": (2, re.compile(r"[01]+\Z"))}


def js_to_string(v: Any) -> str:
    """ToString of a JSON-like value (ECMA-262 7.1.17) as the relational operators' ToPrimitive
    reaches it: arrays join their elements' strings with "," (null / undefined as ""), plain
    objects are "[object Object]"."""
    if v is None or isinstance(v, _Undefined):
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return number_to_js(float(v)) if not (isinstance(v, float) and (math.isnan(v) or math.isinf(v))) else \
            ("NaN" if math.isnan(v) else ("Infinity" if v > 0 else "-Infinity"))
    if isinstance(v, str):
        return v
    if isinstance(v, (list, tuple)):
        return ",".join(js_to_string(e) for e in v)
    return "[object Object]"


def js_to_number(v: Any) -> float:
    """ECMAScript ToNumber (7.1.4) of a JSON-like value, as `length < v` applies it: undefined and
    objects give NaN, null and false 0, true 1, strings by StringToNumber (whitespace trimmed, ""
    is 0, 0x / 0o / 0b literals, "Infinity"; anything else NaN), arrays through their joined
    string ([] is 0, [100] is 100, [1, 2] is NaN)."""
    if isinstance(v, _Undefined):
        return float("nan")
    if v is None:
        return 0.0
    if isinstance(v, bool):
        return 1.0 if v else 0.0
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, (list, tuple)):
        return js_to_number(js_to_string(v))
    if not isinstance(v, str):
        return float("nan")
    t = v.strip(_JS_WS)
    if not t:
        return 0.0
    r = _JS_RADIX.get(t[:2].lower())
    if r is not None:
        return float(int(t[2:], r[0])) if r[1].match(t[2:]) else float("nan")
    if not _JS_DEC.match(t):
        return float("nan")
    return float(t.replace("Infinity", "inf"))
