"""`{{request.object.<path>}}` variables in a rule's validate message (host side).

The device decides statuses; the message of a FAIL / ERROR response is built on the host
(``cli.rule_message``). The reference substitutes the message's variables against the JSON
context in ``buildErrorMessage`` (pkg/engine/validation.go:510-532): ``variables.SubstituteAll``
(vars.go:64-66,173-180) runs the ``$()`` references, then ``substituteVariablesIfAny``
(vars.go:319-398) over the message string, then unescapes ``\\{{``. The context document is
``{"request": {"object": <resource>}}`` re-read with encoding/json, so numbers are float64.

Supported variables: JMESPath field / quoted-field / index chains rooted at ``request.object``
(the only ones ``kyverno apply`` evaluates without ``--set``: common.go:76-80). A missing key, or a
whole-message variable whose value is not a string, makes the reference panic (``msgRaw.(string)``
on a nil / non-string interface, validation.go:519-524); here that raises ``MessageVariableError``.
Other JMESPath forms (projections, pipes, filters, functions) are valid for the reference but not
evaluated here: they raise ``UnsupportedMessageVariable`` (not a reference panic).

``$()`` references in a message resolve against the message string itself (vars.go:253-309,
450-475): the lookup never finds a value, so a plain reference makes SubstituteAll return the
message unchanged together with an error that buildErrorMessage only logs (variables are then not
substituted at all), while an empty or operator-prefixed reference returns nil and panics.
"""
from __future__ import annotations

import decimal
import re

__all__ = ["MessageVariableError", "UnsupportedMessageVariable", "substitute_message", "has_variable",
           "go_json_marshal"]


class MessageVariableError(ValueError):
    """The reference engine panics on this message (unresolvable or non-string substitution)."""


class UnsupportedMessageVariable(ValueError):
    """A message variable the reference evaluates (general JMESPath) that this host does not."""


def _find_vars(s: str) -> list[str]:
    """RegexVariables.FindAllString (vars.go:20): ``^\\{\\{[^{}]*\\}\\}|[^\\\\]\\{\\{[^{}]*\\}\\}``,
    leftmost-first, non-overlapping."""
    out, i, n = [], 0, len(s)

    def close(j):  # end of "{{[^{}]*}}" starting at j, or -1
        if not s.startswith("{{", j):
            return -1
        k = j + 2
        while k < n and s[k] not in "{}":
            k += 1
        return k + 2 if s.startswith("}}", k) else -1

    while i < n:
        if i == 0:
            e = close(0)
            if e >= 0:
                out.append(s[:e])
                i = e
                continue
        if s[i] != "\\":
            e = close(i + 1)
            if e >= 0:
                out.append(s[i:e])
                i = e
                continue
        i += 1
    return out


def has_variable(s: str) -> bool:
    return bool(_find_vars(s))


_REF = re.compile(r"^\$\(.[^ ]*\)|[^\\]\$\(.[^ ]*\)")     # RegexReferences (vars.go:25)
_ESC_REF = re.compile(r"\\\$\(.[^ ]*\)")                  # RegexEscpReferences (vars.go:28)
_TOKEN = re.compile(r'\.?([A-Za-z_][A-Za-z0-9_]*)|\.?"((?:[^"\\]|\\.)*)"|\[(-?\d+)\]')


def _query(expr: str, context) -> object:
    """ctx.Query (pkg/engine/context/evaluate.go:15-50) for field / quoted-field / index chains."""
    expr = expr.strip()
    pos, cur = 0, context
    steps = []
    while pos < len(expr):
        m = _TOKEN.match(expr, pos)
        if not m or (pos == 0 and expr[0] in ".["):
            raise UnsupportedMessageVariable(f"JMESPath expression not evaluated here: {expr!r}")
        steps.append(m)
        pos = m.end()
    if not steps:
        raise MessageVariableError("invalid query (nil)")
    for m in steps:
        if m.group(3) is not None:
            if not isinstance(cur, list):
                cur = None
                continue
            i = int(m.group(3))
            cur = cur[i] if -len(cur) <= i < len(cur) else None
            continue
        key = m.group(1) if m.group(1) is not None else re.sub(r"\\(.)", r"\1", m.group(2))
        if isinstance(cur, dict):
            if key not in cur:
                raise MessageVariableError(f'Unknown key "{key}" in path')
            cur = cur[key]
        else:
            cur = None
    return cur


def _operator(p: str) -> str:
    """operator.GetOperatorFromStringPattern (pkg/engine/operator/operator.go:33-67)."""
    if len(p) < 2:
        return ""
    for op in (">=", "<=", ">", "<", "!"):
        if p.startswith(op):
            return op
    # RE2: \d is ASCII, $ is the end of the text
    if re.match(r"([0-9]+(\.[0-9]+)?)([^-]*)!-([0-9]+(\.[0-9]+)?)([^-]*)\Z", p):
        return "!-"
    if re.match(r"([0-9]+(\.[0-9]+)?)([^-]*)-([0-9]+(\.[0-9]+)?)([^-]*)\Z", p):
        return "-"
    return ""


def _go_float(f: float) -> str:
    """encoding/json float64 encoding: strconv 'f' -1, or 'e' -1 outside [1e-6, 1e21) with the
    exponent's leading zero dropped (encode.go floatEncoder)."""
    a = abs(f)
    if a != 0 and (a < 1e-6 or a >= 1e21):
        s = repr(f)
        if "e" not in s:
            s = "%e" % f
        m = re.match(r"^(-?[\d.]+)e([+-])(\d+)$", s)
        mant, sign, exp = m.group(1), m.group(2), m.group(3)
        if len(exp) == 1:
            exp = "0" + exp
        if sign == "-" and len(exp) == 2 and exp[0] == "0":
            exp = exp[1:]
        return f"{mant}e{sign}{exp}"
    d = decimal.Decimal(repr(f)).normalize()
    return format(d, "f")


def _go_json_string(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_json_marshal(v) -> str:
    """json.Marshal of an encoding/json-decoded value (map keys sorted, HTML-safe escaping)."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, (int, float)):
        return _go_float(float(v))
    if isinstance(v, str):
        return _go_json_string(v)
    if isinstance(v, list):
        return "[" + ",".join(go_json_marshal(x) for x in v) + "]"
    if isinstance(v, dict):
        keys = sorted(v, key=lambda k: k.encode("utf-8"))
        return "{" + ",".join(_go_json_string(k) + ":" + go_json_marshal(v[k]) for k in keys) + "}"
    raise MessageVariableError(f"failed to marshal {type(v).__name__}")


def substitute_message(msg: str, resource: dict) -> str:
    """The message after SubstituteAll with context ``request.object = resource``: references
    (vars.go:253-309), then substituteVariablesIfAny (vars.go:319-398), then ``\\{{`` unescaping."""
    context = {"request": {"object": resource}}
    # substituteReferencesIfAny on the message document (vars.go:253-309): the first reference
    # decides. resolveReference (vars.go:450-475) looks the path up in the message string itself,
    # whose only leaf sits at path "", so nothing is ever found: an empty path errors (nil element:
    # panic), an operator fails valFromReferenceToString(nil) (nil element: panic), a plain
    # reference resolves to nil and returns the original string with an error that
    # buildErrorMessage only logs (validation.go:519-522) -- no variable substitution follows
    m = _REF.search(msg)
    if m:
        v = m.group(0)
        if not v.startswith("$("):
            v = v[1:]
        path = v.strip("$()")
        op = _operator(path)
        path = path[len(op):]
        if not path:
            raise MessageVariableError(f"empty $() reference in message {msg!r}")
        if op:
            raise MessageVariableError(f"$() reference with operator {op!r} in message {msg!r} resolves to nil")
        return msg
    value = _ESC_REF.sub(lambda m: m.group(0)[1:], msg)
    vs = _find_vars(value)
    while vs:
        original = value
        for v in vs:
            initial = v.startswith("{{")
            old = v
            if not initial:
                v = v[1:]
            variable = v.replace("{{", "").replace("}}", "").strip()
            if variable == "@":
                raise MessageVariableError("'@' in a message has no pattern path (getJMESPath panics)")
            got = _query(variable, context)
            if original == v:
                if not isinstance(got, str):
                    raise MessageVariableError(f"message {msg!r} resolves to a non-string {type(got).__name__}")
                return got
            prefix = "" if initial else old[0]
            sub = got if isinstance(got, str) else go_json_marshal(got)
            # substituteVarInPattern(prefix, originalPattern, ...): each substitution of a round
            # starts from the round's original string; the outer loop picks up what is left
            value = original.replace(prefix + v, prefix + sub, 1)
        vs = _find_vars(value)
    # RegexEscpVariables: \{{...}} -> {{...}}
    return re.sub(r"\\(\{\{[^{}]*\}\})", r"\1", value)
