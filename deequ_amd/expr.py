"""Compile deequ's Spark SQL predicate strings into the dq_predicate postfix program (include/dq.h).

deequ passes `where` filters and Compliance predicates as Spark SQL expression strings
(`expr(...)` in A/Analyzer.scala:409-432 and A/Compliance.scala:49-52; generated ones in
M/checks/Check.scala:594-943). This module parses Spark SQL's scalar expression language over one row —
comparisons (= == != <> < <= > >= <=>), IN, IS [NOT] NULL, [NOT] LIKE, [NOT] RLIKE / REGEXP (java.util.regex
through deequ_amd/regex.py), [NOT] BETWEEN, AND / OR / NOT, + - * / %, CASE WHEN .. THEN .. [ELSE ..] END (searched
and simple forms), CAST, DATE 'yyyy-MM-dd' literals and the functions coalesce / nvl / ifnull, if, isnull /
isnotnull, isnan, nanvl, abs, length, lower / lcase, upper / ucase, trim / ltrim / rtrim, substring / substr,
year / month / dayofmonth / day — resolving column names against the table schema exactly like Spark's analyzer
would: an unknown column raises (Spark's AnalysisException), which the runner turns into a failure of every
shareable analyzer of the batch (R/AnalysisRunner.scala:320-323). Anything else raises PredicateSyntaxError.
"""
import ctypes
import re

import numpy as np

from . import native as N


class PredicateSyntaxError(ValueError):
    """Unparseable predicate (Spark: ParseException)."""


class UnresolvedColumnError(ValueError):
    """Predicate references a column the data does not have (Spark: AnalysisException)."""


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>\d+\.\d*(?:[eE][+-]?\d+)?[dD]?|\.\d+(?:[eE][+-]?\d+)?[dD]?|\d+(?:[eE][+-]?\d+)?[dDlL]?)
  | (?P<str>'(?:[^'\\]|\\.|'')*'|"(?:[^"\\]|\\.)*")
  | (?P<bq>`[^`]+`)
  | (?P<op><=>|<=|>=|<>|!=|==|=|<|>|\+|-|\*|/|%|\(|\)|,)
  | (?P<id>[A-Za-z_][A-Za-z0-9_.]*)
""", re.VERBOSE)

_KEYWORDS = {"AND", "OR", "NOT", "IS", "NULL", "IN", "LIKE", "TRUE", "FALSE", "BETWEEN", "CAST", "AS", "RLIKE",
             "REGEXP", "CASE", "WHEN", "THEN", "ELSE", "END", "DATE"}


def _tokenize(text):
    pos, out = 0, []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise PredicateSyntaxError("cannot parse predicate %r at %d" % (text, pos))
        pos = m.end()
        kind = m.lastgroup
        val = m.group(kind)
        if kind == "ws":
            continue
        if kind == "id" and val.upper() in _KEYWORDS:
            out.append(("kw", val.upper()))
        elif kind == "bq":
            out.append(("id", val[1:-1]))
        elif kind == "str":
            body = val[1:-1]
            if val[0] == "'":
                body = body.replace("''", "'")
            body = re.sub(r"\\(.)", lambda mm: {"n": "\n", "t": "\t"}.get(mm.group(1), mm.group(1)), body)
            out.append(("str", body))
        else:
            out.append((kind, val))
    out.append(("eof", None))
    return out


class _Node:
    def __init__(self, kind, *children, value=None):
        self.kind, self.children, self.value = kind, list(children), value


class _Parser:
    """Recursive descent with Spark SQL precedence: OR < AND < NOT < predicate < + - < * / % < unary."""

    def __init__(self, text):
        self.toks = _tokenize(text)
        self.i = 0
        self.text = text

    def peek(self, k=0):
        return self.toks[self.i + k]

    def take(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, val=None):
        t = self.peek()
        if t[0] == kind and (val is None or t[1] == val):
            self.i += 1
            return True
        return False

    def expect(self, kind, val=None):
        if not self.accept(kind, val):
            raise PredicateSyntaxError("expected %s in %r, got %r" % (val or kind, self.text, self.peek()[1]))

    def parse(self):
        n = self.or_()
        if self.peek()[0] != "eof":
            raise PredicateSyntaxError("trailing input in %r near %r" % (self.text, self.peek()[1]))
        return n

    def or_(self):
        n = self.and_()
        while self.accept("kw", "OR"):
            n = _Node("or", n, self.and_())
        return n

    def and_(self):
        n = self.not_()
        while self.accept("kw", "AND"):
            n = _Node("and", n, self.not_())
        return n

    def not_(self):
        if self.accept("kw", "NOT"):
            return _Node("not", self.not_())
        return self.pred()

    def pred(self):
        left = self.add()
        t = self.peek()
        if t[0] == "op" and t[1] in ("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
            self.take()
            op = {"==": "=", "<>": "!="}.get(t[1], t[1])
            return _Node("cmp", left, self.add(), value=op)
        negate = False
        if t == ("kw", "NOT") and self.peek(1)[0] == "kw" and self.peek(1)[1] in ("IN", "LIKE", "BETWEEN", "RLIKE",
                                                                                   "REGEXP"):
            self.take()
            negate = True
            t = self.peek()
        if self.accept("kw", "IS"):
            neg = self.accept("kw", "NOT")
            self.expect("kw", "NULL")
            return _Node("isnotnull" if neg else "isnull", left)
        if self.accept("kw", "IN"):
            self.expect("op", "(")
            items = [self.add()]
            while self.accept("op", ","):
                items.append(self.add())
            self.expect("op", ")")
            n = _Node("in", left, *items)
            return _Node("not", n) if negate else n
        if self.accept("kw", "LIKE"):
            pat = self.take()
            if pat[0] != "str":
                raise PredicateSyntaxError("LIKE needs a string literal pattern in %r" % self.text)
            n = _Node("like", left, value=pat[1])
            return _Node("not", n) if negate else n
        if self.accept("kw", "RLIKE") or self.accept("kw", "REGEXP"):
            pat = self.take()
            if pat[0] != "str":
                raise PredicateSyntaxError("RLIKE needs a string literal pattern in %r" % self.text)
            n = _Node("rlike", left, value=pat[1])
            return _Node("not", n) if negate else n
        if self.accept("kw", "BETWEEN"):
            lo = self.add()
            self.expect("kw", "AND")
            hi = self.add()
            n = _Node("and", _Node("cmp", left, lo, value=">="), _Node("cmp", left, hi, value="<="))
            return _Node("not", n) if negate else n
        return left

    def add(self):
        n = self.mul()
        while self.peek()[0] == "op" and self.peek()[1] in ("+", "-"):
            op = self.take()[1]
            n = _Node("arith", n, self.mul(), value=op)
        return n

    def mul(self):
        n = self.unary()
        while self.peek()[0] == "op" and self.peek()[1] in ("*", "/", "%"):
            op = self.take()[1]
            n = _Node("arith", n, self.unary(), value=op)
        return n

    def unary(self):
        if self.accept("op", "-"):
            return _Node("neg", self.unary())
        if self.accept("op", "+"):
            return self.unary()
        return self.atom()

    def atom(self):
        t = self.take()
        kind, val = t
        if kind == "op" and val == "(":
            n = self.or_()
            self.expect("op", ")")
            return n
        if kind == "num":
            v = val.rstrip("dDlL")
            if re.fullmatch(r"\d+", v) and not val[-1:] in "dD":
                return _Node("const", value=("long", int(v)))
            return _Node("const", value=("double", float(v)))
        if kind == "str":
            return _Node("const", value=("string", val))
        if kind == "kw" and val in ("TRUE", "FALSE"):
            return _Node("const", value=("bool", val == "TRUE"))
        if kind == "kw" and val == "NULL":
            return _Node("null")
        if kind == "kw" and val == "DATE":  # DATE 'yyyy-MM-dd' literal: days since the epoch (a DATE column's value)
            lit = self.take()
            if lit[0] != "str":
                raise PredicateSyntaxError("DATE needs a string literal in %r" % self.text)
            return _Node("const", value=("long", _date_days(lit[1], self.text)))
        if kind == "kw" and val == "CASE":
            return self._case()
        if kind == "kw" and val == "CAST":
            self.expect("op", "(")
            e = self.or_()
            self.expect("kw", "AS")
            ty = self.take()
            if ty[0] != "id":
                raise PredicateSyntaxError("bad CAST target in %r" % self.text)
            tname = ty[1].lower()
            if self.accept("op", "("):  # decimal(p,s)
                while not self.accept("op", ")"):
                    self.take()
            self.expect("op", ")")
            if tname in ("double", "float", "decimal"):
                return _Node("cast_double", e)
            if tname in ("int", "integer", "long", "bigint", "short", "smallint", "tinyint", "byte"):
                return _Node("cast_long", e)
            if tname in ("string",):
                return e
            raise PredicateSyntaxError("unsupported CAST target %s" % tname)
        if kind == "id":
            if self.accept("op", "("):
                fname = val.lower()
                args = []
                if not self.accept("op", ")"):
                    args.append(self.or_())
                    while self.accept("op", ","):
                        args.append(self.or_())
                    self.expect("op", ")")
                n = self._function(fname, args)
                if n is None:
                    raise PredicateSyntaxError("unsupported function %s/%d in %r" % (val, len(args), self.text))
                return n
            return _Node("col", value=val)
        raise PredicateSyntaxError("unexpected %r in %r" % (val, self.text))


    _UNARY = {"length": "length", "char_length": "length", "character_length": "length", "isnull": "isnull",
              "isnotnull": "isnotnull", "isnan": "isnan", "abs": "abs", "lower": "lower", "lcase": "lower",
              "upper": "upper", "ucase": "upper", "trim": "trim", "ltrim": "ltrim", "rtrim": "rtrim", "year": "year",
              "month": "month", "dayofmonth": "day", "day": "day"}

    def _function(self, fname, args):
        if fname == "coalesce" and args:
            return _Node("coalesce", *args)
        if fname in ("nvl", "ifnull") and len(args) == 2:
            return _Node("coalesce", *args)
        if fname == "if" and len(args) == 3:  # if(c, a, b) = CASE WHEN c THEN a ELSE b END
            return _Node("case", args[0], args[1], args[2], value=(1, True))
        if fname == "nanvl" and len(args) == 2:
            return _Node("nanvl", *args)
        if fname in ("substring", "substr") and len(args) in (2, 3):
            if len(args) == 2:
                args.append(_Node("const", value=("long", 2147483647)))
            return _Node("substr", *args)
        if fname in self._UNARY and len(args) == 1:
            return _Node(self._UNARY[fname], args[0])
        return None

    def _case(self):
        """CASE [x] WHEN w THEN v ... [ELSE e] END; the simple form's WHEN w means x = w."""
        subject = None
        if self.peek() != ("kw", "WHEN"):
            subject = self.or_()
        parts = []
        while self.accept("kw", "WHEN"):
            cond = self.or_()
            if subject is not None:
                cond = _Node("cmp", subject, cond, value="=")
            self.expect("kw", "THEN")
            parts += [cond, self.or_()]
        if not parts:
            raise PredicateSyntaxError("CASE without WHEN in %r" % self.text)
        has_else = self.accept("kw", "ELSE")
        if has_else:
            parts.append(self.or_())
        self.expect("kw", "END")
        return _Node("case", *parts, value=(len(parts) // 2, has_else))


def _date_days(text, where):
    """DATE 'yyyy-MM-dd' as days since 1970-01-01 (proleptic Gregorian, Spark's DateTimeUtils.stringToDate for dates
    after the 1582 cutover)."""
    import datetime
    m = re.fullmatch(r"\s*(\d{4})-(\d{1,2})-(\d{1,2})\s*", text)
    if not m:
        raise PredicateSyntaxError("bad DATE literal %r in %r" % (text, where))
    d = datetime.date(int(m.group(1)), int(m.group(2)), int(m.group(3)))
    return (d - datetime.date(1970, 1, 1)).days


class CompiledPredicate:
    """Postfix program + constant pool; keeps the ctypes buffers alive while referenced."""

    def __init__(self, text, code, consts, strings, columns):
        self.text = text
        self.columns = columns
        self._code = np.asarray(code, dtype=np.int32)
        self._consts = (N.DqConst * max(len(consts), 1))(*consts)
        self._n_consts = len(consts)
        self._strings = np.frombuffer(bytes(strings) or b"\0", dtype=np.uint8).copy()
        self._strings_len = len(strings)

    def to_native(self):
        p = N.DqPredicate()
        p.code = self._code.ctypes.data
        p.code_len = len(self._code)
        p.n_consts = self._n_consts
        p.consts = ctypes.cast(self._consts, ctypes.c_void_p)
        p.strings = self._strings.ctypes.data
        p.strings_len = self._strings_len
        return p


_CMP = {"=": N.P_EQ, "!=": N.P_NE, "<": N.P_LT, "<=": N.P_LE, ">": N.P_GT, ">=": N.P_GE, "<=>": N.P_EQ_NULLSAFE}
_ARITH = {"+": N.P_ADD, "-": N.P_SUB, "*": N.P_MUL, "/": N.P_DIV, "%": N.P_MOD}


def compile_predicate(text, column_index, column_types=None):
    """`column_index`: name -> index into the batch's column list; `column_types`: name -> Spark type (for the
    functions whose meaning depends on it: year / month / day of a DATE or a TIMESTAMP). Returns CompiledPredicate."""
    tree = _Parser(text).parse()
    code, consts, strings, used = [], [], bytearray(), []
    column_types = column_types or {}

    def resolve(name):
        if name in column_index:
            return name
        # Spark resolves identifiers case-insensitively by default.
        matches = [c for c in column_index if c.lower() == name.lower()]
        if len(matches) != 1:
            raise UnresolvedColumnError("cannot resolve '`%s`' given input columns: [%s]"
                                        % (name, ", ".join(column_index)))
        return matches[0]

    def blob_const(image):
        """A STRING constant holding a binary image, 4-byte aligned in the pool (regex programs)."""
        while len(strings) % 4:
            strings.append(0)
        c = N.DqConst()
        c.tag, c.str_offset, c.str_len = N.V_STRING, len(strings), len(image)
        strings.extend(image)
        consts.append(c)
        return len(consts) - 1

    def const(kind, v):
        c = N.DqConst()
        if kind == "long":
            c.tag, c.i64 = N.V_LONG, int(v)
        elif kind == "double":
            c.tag, c.f64 = N.V_DOUBLE, float(v)
        elif kind == "bool":
            c.tag, c.i64 = N.V_BOOL, 1 if v else 0
        else:
            b = v.encode("utf-8")
            c.tag, c.str_offset, c.str_len = N.V_STRING, len(strings), len(b)
            strings.extend(b)
        consts.append(c)
        return len(consts) - 1

    def emit(n):
        k = n.kind
        if k == "col":
            name = resolve(n.value)
            code.extend([N.P_COL, column_index[name]])
            used.append(name)
        elif k == "const":
            code.extend([N.P_CONST, const(*n.value)])
        elif k == "null":
            code.extend([N.P_NULL, 0])
        elif k == "cmp":
            emit(n.children[0])
            emit(n.children[1])
            code.extend([_CMP[n.value], 0])
        elif k in ("and", "or"):
            emit(n.children[0])
            emit(n.children[1])
            code.extend([N.P_AND if k == "and" else N.P_OR, 0])
        elif k == "not":
            emit(n.children[0])
            code.extend([N.P_NOT, 0])
        elif k in ("isnull", "isnotnull"):
            emit(n.children[0])
            code.extend([N.P_IS_NULL if k == "isnull" else N.P_IS_NOT_NULL, 0])
        elif k == "in":
            for ch in n.children:
                emit(ch)
            code.extend([N.P_IN, len(n.children) - 1])
        elif k == "coalesce":
            for ch in n.children:
                emit(ch)
            code.extend([N.P_COALESCE, len(n.children)])
        elif k == "arith":
            emit(n.children[0])
            emit(n.children[1])
            code.extend([_ARITH[n.value], 0])
        elif k == "neg":
            emit(n.children[0])
            code.extend([N.P_NEG, 0])
        elif k in ("abs", "isnan", "lower", "upper"):
            emit(n.children[0])
            code.extend([{"abs": N.P_ABS, "isnan": N.P_ISNAN, "lower": N.P_LOWER, "upper": N.P_UPPER}[k], 0])
        elif k in ("trim", "ltrim", "rtrim"):
            emit(n.children[0])
            code.extend([N.P_TRIM, {"trim": 0, "ltrim": 1, "rtrim": 2}[k]])
        elif k == "nanvl":
            emit(n.children[0])
            emit(n.children[1])
            code.extend([N.P_NANVL, 0])
        elif k == "substr":
            for ch in n.children:
                emit(ch)
            code.extend([N.P_SUBSTR, 0])
        elif k == "case":
            nwhen, has_else = n.value
            for ch in n.children:
                emit(ch)
            code.extend([N.P_CASE, 2 * nwhen + (1 if has_else else 0)])
        elif k == "rlike":
            from .regex import compile_regex
            emit(n.children[0])
            code.extend([N.P_RLIKE, blob_const(compile_regex(n.value).to_bytes())])
        elif k in ("year", "month", "day"):
            child = n.children[0]
            ty = column_types.get(resolve(child.value)) if child.kind == "col" else None
            if ty not in (N.TYPE_DATE, N.TYPE_TIMESTAMP):
                raise PredicateSyntaxError("%s() needs a DATE or TIMESTAMP column in %r" % (k, text))
            emit(child)
            code.extend([{"year": N.P_YEAR, "month": N.P_MONTH, "day": N.P_DAY}[k],
                         1 if ty == N.TYPE_TIMESTAMP else 0])
        elif k == "like":
            emit(n.children[0])
            code.extend([N.P_LIKE, const("string", n.value)])
        elif k == "length":
            emit(n.children[0])
            code.extend([N.P_LENGTH, 0])
        elif k == "cast_double":
            emit(n.children[0])
            code.extend([N.P_CAST_DOUBLE, 0])
        elif k == "cast_long":
            emit(n.children[0])
            code.extend([N.P_CAST_LONG, 0])
        else:
            raise PredicateSyntaxError("unsupported node %s" % k)

    emit(tree)
    return CompiledPredicate(text, code, consts, strings, used)


def referenced_columns(text):
    """Column names a predicate reads (for schema checks without compiling)."""
    return [t[1] for t in _tokenize(text) if t[0] == "id"]
