"""java.util.regex subset -> backtracking bytecode for the GPU (PatternMatch, A/PatternMatch.scala:37-55).

deequ's PatternMatch counts rows where `regexp_extract(col, pattern, 0) != ""` (:46-48), i.e. where
the FIRST match java.util.regex.Matcher.find() reports is non-empty. Java's matcher is a
backtracking engine with leftmost-first priorities; the GPU runs the same kind of engine (one lane
per row, deequ_amd/csrc/regex.hip), so this module only parses the pattern and emits its program.

Supported (everything deequ's Patterns — EMAIL, URL, SOCIAL_SECURITY_NUMBER_US, CREDITCARD,
A/PatternMatch.scala:57-72 — and the reference tests use): literals and escapes (\\t \\n \\r \\f \\e
\\a \\xhh \\uhhhh \\0oo, escaped metacharacters), `.`, classes with ranges / negation / nested
escapes, \\d \\D \\s \\S \\w \\W (ASCII, Java's defaults), groups (capturing, (?:...)), lookahead
(?=...) (?!...), alternation, greedy and lazy quantifiers * + ? {n} {n,} {n,m}, anchors ^ $ \\b \\B
\\A \\z \\Z (no MULTILINE), backreferences \\1..\\9. Unsupported constructs (flags, possessive or
atomic groups, lookbehind, named groups, class intersections, Unicode properties) raise
`RegexUnsupported`, which the analyzer reports as a failed metric — there is no CPU fallback.
"""
import struct

# opcodes (deequ_amd/csrc/regex.hip)
OP_CHAR, OP_CLASS, OP_ANY, OP_SPLIT, OP_JMP, OP_SAVE, OP_ASSERT, OP_BACKREF, OP_LOOK, OP_LOOKEND, OP_MARK, \
    OP_CHECK, OP_MATCH = range(1, 14)
A_BOL, A_EOL, A_WORDB, A_NWORDB, A_BEGIN, A_END, A_ENDZ = range(7)
MAX_CP = 0x10FFFF
MAGIC = 0x52454758  # "REGX"


from .metrics import UnsupportedOnDevice


class RegexUnsupported(UnsupportedOnDevice):
    pass


# ---- parser -> AST --------------------------------------------------------------------------------
# nodes: ("char", cp) ("class", ranges) ("any",) ("cat", [..]) ("alt", [..]) ("group", idx|None, node)
#        ("rep", node, min, max|None, greedy) ("assert", kind) ("backref", n) ("look", neg, node)

DIGIT = [(48, 57)]
SPACE = [(9, 13), (32, 32)]  # [ \t\n\x0B\f\r]
WORD = [(48, 57), (65, 90), (95, 95), (97, 122)]


def _normalize(ranges):
    out = []
    for lo, hi in sorted(ranges):
        if out and lo <= out[-1][1] + 1:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def _negate(ranges):
    out, prev = [], 0
    for lo, hi in _normalize(ranges):
        if lo > prev:
            out.append((prev, lo - 1))
        prev = hi + 1
    if prev <= MAX_CP:
        out.append((prev, MAX_CP))
    return out


class _Parser:
    def __init__(self, pattern):
        self.p = pattern
        self.i = 0
        self.ngroups = 0

    def peek(self, k=0):
        j = self.i + k
        return self.p[j] if j < len(self.p) else None

    def take(self):
        c = self.p[self.i]
        self.i += 1
        return c

    def parse(self):
        node = self.alt()
        if self.i != len(self.p):
            raise RegexUnsupported("unbalanced ')' at %d" % self.i)
        return node

    def alt(self):
        branches = [self.cat()]
        while self.peek() == "|":
            self.take()
            branches.append(self.cat())
        return branches[0] if len(branches) == 1 else ("alt", branches)

    def cat(self):
        items = []
        while self.peek() is not None and self.peek() not in "|)":
            items.append(self.repeat())
        return ("cat", items)

    def repeat(self):
        atom = self.atom()
        while True:
            c = self.peek()
            if c in ("*", "+", "?"):
                self.take()
                lo, hi = {"*": (0, None), "+": (1, None), "?": (0, 1)}[c]
            elif c == "{" and self._is_counted():
                lo, hi = self._counted()
            else:
                return atom
            greedy = True
            if self.peek() == "?":
                self.take()
                greedy = False
            elif self.peek() == "+":
                raise RegexUnsupported("possessive quantifiers are not supported")
            if atom[0] in ("assert", "look"):
                raise RegexUnsupported("quantified assertion")
            atom = ("rep", atom, lo, hi, greedy)

    def _is_counted(self):
        j = self.i + 1
        while j < len(self.p) and (self.p[j].isdigit() or self.p[j] == ","):
            j += 1
        return j < len(self.p) and self.p[j] == "}" and j > self.i + 1 and self.p[self.i + 1].isdigit()

    def _counted(self):
        self.take()
        body = ""
        while self.peek() != "}":
            body += self.take()
        self.take()
        if "," in body:
            a, b = body.split(",", 1)
            return int(a), (int(b) if b else None)
        return int(body), int(body)

    def atom(self):
        c = self.take()
        if c == "(":
            if self.peek() == "?":
                self.take()
                k = self.take()
                if k == ":":
                    node = ("group", None, self.alt())
                elif k in ("=", "!"):
                    node = ("look", k == "!", self.alt())
                else:
                    raise RegexUnsupported("group construct (?%s is not supported" % k)
            else:
                self.ngroups += 1
                idx = self.ngroups
                node = ("group", idx, self.alt())
            if self.peek() != ")":
                raise RegexUnsupported("missing ')'")
            self.take()
            return node
        if c == "[":
            return ("class", self._class())
        if c == ".":
            return ("any",)
        if c == "^":
            return ("assert", A_BOL)
        if c == "$":
            return ("assert", A_EOL)
        if c == "\\":
            return self._escape(in_class=False)
        if c in ")*+?{":
            raise RegexUnsupported("dangling metacharacter %r" % c)  # Java: "Dangling meta character" / "Illegal repetition"
        return ("char", ord(c))

    def _escape(self, in_class):
        c = self.take()
        simple = {"t": 9, "n": 10, "r": 13, "f": 12, "e": 27, "a": 7}
        if c in simple:
            return ("char", simple[c])
        if c == "x":
            h = self.take() + self.take()
            return ("char", int(h, 16))
        if c == "u":
            h = "".join(self.take() for _ in range(4))
            return ("char", int(h, 16))
        if c == "0":
            o = ""
            while len(o) < 3 and self.peek() is not None and self.peek() in "01234567":
                o += self.take()
            return ("char", int(o or "0", 8))
        if c == "d":
            return ("class", DIGIT)
        if c == "D":
            return ("class", _negate(DIGIT))
        if c == "s":
            return ("class", SPACE)
        if c == "S":
            return ("class", _negate(SPACE))
        if c == "w":
            return ("class", WORD)
        if c == "W":
            return ("class", _negate(WORD))
        if not in_class:
            if c == "b":
                return ("assert", A_WORDB)
            if c == "B":
                return ("assert", A_NWORDB)
            if c == "A":
                return ("assert", A_BEGIN)
            if c == "z":
                return ("assert", A_END)
            if c == "Z":
                return ("assert", A_ENDZ)
            if c.isdigit():
                return ("backref", int(c))
        if c.isalpha():
            raise RegexUnsupported("escape \\%s is not supported" % c)
        return ("char", ord(c))

    def _class(self):
        neg = False
        if self.peek() == "^":
            self.take()
            neg = True
        ranges = []
        first = True
        while True:
            c = self.peek()
            if c is None:
                raise RegexUnsupported("unterminated character class")
            if c == "]" and not first:
                self.take()
                break
            first = False
            if c == "[":
                raise RegexUnsupported("nested classes / intersections are not supported")
            if c == "&" and self.peek(1) == "&":
                raise RegexUnsupported("class intersections are not supported")
            lo = self._class_atom()
            if lo[0] == "class":
                ranges.extend(lo[1])
                continue
            lo = lo[1]
            if self.peek() == "-" and self.peek(1) not in (None, "]"):
                self.take()
                hi = self._class_atom()
                if hi[0] == "class":
                    raise RegexUnsupported("illegal character range")
                ranges.append((lo, hi[1]))
            else:
                ranges.append((lo, lo))
        ranges = _normalize(ranges)
        return _negate(ranges) if neg else ranges

    def _class_atom(self):
        c = self.take()
        if c == "\\":
            return self._escape(in_class=True)
        return ("char", ord(c))


# ---- AST -> bytecode ------------------------------------------------------------------------------
class _Emitter:
    def __init__(self):
        self.code = []  # [op, a, b]
        self.classes = []
        self.nloops = 0

    def emit(self, op, a=0, b=0):
        self.code.append([op, a, b])
        return len(self.code) - 1

    def cls(self, ranges):
        self.classes.append(_normalize(ranges))
        return len(self.classes) - 1

    def gen(self, n):
        k = n[0]
        if k == "char":
            self.emit(OP_CHAR, n[1])
        elif k == "class":
            self.emit(OP_CLASS, self.cls(n[1]))
        elif k == "any":
            self.emit(OP_ANY)
        elif k == "cat":
            for x in n[1]:
                self.gen(x)
        elif k == "alt":
            jumps = []
            for j, br in enumerate(n[1]):
                if j < len(n[1]) - 1:
                    split = self.emit(OP_SPLIT)
                    self.code[split][1] = len(self.code)
                    self.gen(br)
                    jumps.append(self.emit(OP_JMP))
                    self.code[split][2] = len(self.code)
                else:
                    self.gen(br)
            for jp in jumps:
                self.code[jp][1] = len(self.code)
        elif k == "group":
            if n[1] is None:
                self.gen(n[2])
            else:
                self.emit(OP_SAVE, 2 * n[1])
                self.gen(n[2])
                self.emit(OP_SAVE, 2 * n[1] + 1)
        elif k == "assert":
            self.emit(OP_ASSERT, n[1])
        elif k == "backref":
            self.emit(OP_BACKREF, n[1])
        elif k == "look":
            look = self.emit(OP_LOOK, 0, 1 if n[1] else 0)
            self.gen(n[2])
            self.emit(OP_LOOKEND)
            self.code[look][1] = len(self.code)
        elif k == "rep":
            _, body, lo, hi, greedy = n
            for _ in range(lo):
                self.gen(body)
            if hi is None:
                self._star(body, greedy)
            else:
                self._optional_chain(body, hi - lo, greedy)
        else:
            raise RegexUnsupported(k)

    def _star(self, body, greedy):
        nullable = _nullable(body)
        loop = self.nloops if nullable else -1
        if nullable:
            self.nloops += 1
        top = self.emit(OP_SPLIT)
        body_start = len(self.code)
        if nullable:
            self.emit(OP_MARK, loop)
        self.gen(body)
        if nullable:
            self.emit(OP_CHECK, loop)  # an empty iteration does not loop again
        self.emit(OP_JMP, top)
        exit_pc = len(self.code)
        self.code[top][1], self.code[top][2] = (body_start, exit_pc) if greedy else (exit_pc, body_start)

    def _optional_chain(self, body, count, greedy):
        splits = []
        for _ in range(count):
            s = self.emit(OP_SPLIT)
            splits.append(s)
            self.code[s][1 if greedy else 2] = len(self.code)
            self.gen(body)
        end = len(self.code)
        for s in splits:
            self.code[s][2 if greedy else 1] = end


def _nullable(n):
    k = n[0]
    if k in ("char", "class", "any", "backref"):
        return k == "backref"
    if k in ("assert", "look"):
        return True
    if k == "cat":
        return all(_nullable(x) for x in n[1])
    if k == "alt":
        return any(_nullable(x) for x in n[1])
    if k == "group":
        return _nullable(n[2])
    if k == "rep":
        return n[2] == 0 or _nullable(n[1])
    return True


class CompiledRegex:
    def __init__(self, pattern, code, classes, ngroups, nloops, anchored):
        self.pattern, self.code, self.classes = pattern, code, classes
        self.ngroups, self.nloops, self.anchored = ngroups, nloops, anchored

    def to_bytes(self):
        """Program image read by regex.hip: header, instructions (3 x int32), class table
        (offset, count) and ranges (lo, hi) — all little-endian int32."""
        nranges = sum(len(c) for c in self.classes)
        header = [MAGIC, len(self.code), len(self.classes), nranges, self.ngroups, self.nloops,
                  1 if self.anchored else 0, 0]
        words = list(header)
        for op, a, b in self.code:
            words += [op, a, b]
        off = 0
        for c in self.classes:
            words += [off, len(c)]
            off += len(c)
        for c in self.classes:
            for lo, hi in c:
                words += [lo, hi]
        return struct.pack("<%di" % len(words), *words)


MAX_GROUPS = 9
MAX_LOOPS = 16
MAX_INSTRUCTIONS = 4096


def compile_regex(pattern):
    p = _Parser(pattern)
    ast = p.parse()
    if p.ngroups > MAX_GROUPS:
        raise RegexUnsupported("more than %d capturing groups" % MAX_GROUPS)
    _check_backrefs(ast, p.ngroups)
    e = _Emitter()
    e.gen(ast)
    e.emit(OP_MATCH)
    if e.nloops > MAX_LOOPS:
        raise RegexUnsupported("too many nullable loops")
    if len(e.code) > MAX_INSTRUCTIONS:
        raise RegexUnsupported("pattern too large")
    anchored = ast[0] == "cat" and ast[1] and ast[1][0] == ("assert", A_BOL)
    return CompiledRegex(pattern, e.code, e.classes, p.ngroups, e.nloops, anchored)


def _check_backrefs(n, ngroups):
    if n[0] == "backref" and n[1] > ngroups:
        raise RegexUnsupported("backreference to undefined group %d" % n[1])
    for x in n[1:]:
        if isinstance(x, tuple):
            _check_backrefs(x, ngroups)
        elif isinstance(x, list):
            for y in x:
                if isinstance(y, tuple):
                    _check_backrefs(y, ngroups)
