"""java.util.regex -> backtracking bytecode for the GPU (PatternMatch, A/PatternMatch.scala:37-55).

deequ's PatternMatch counts rows where `regexp_extract(col, pattern, 0) != ""` (:46-48), i.e. where
the FIRST match java.util.regex.Matcher.find() reports is non-empty. Java's matcher is a
backtracking engine with leftmost-first priorities; the GPU runs the same kind of engine (one lane
per row, deequ_amd/csrc/regex.hip), so this module only parses the pattern and emits its program.

Supported — the java.util.regex (Java 8) syntax:
  * literals and escapes (\\t \\n \\r \\f \\e \\a \\xhh \\x{h..h} \\uhhhh \\0oo \\cX, escaped metacharacters,
    \\Q...\\E quoting), `.`, classes with ranges / negation / nested escapes, nested classes (union,
    `[a-d[m-p]]`) and intersections (`[a-z&&[^aeiou]]`);
  * \\d \\D \\s \\S \\w \\W (ASCII, Java's defaults), \\h \\H \\v \\V (Java 8 horizontal / vertical
    whitespace), \\R (a linebreak);
  * POSIX / java.lang.Character / Unicode properties \\p{..} \\P{..} \\pL: Lower Upper ASCII Alpha Digit
    Alnum Punct Graph Print Blank Cntrl XDigit Space (US-ASCII, as Java without UNICODE_CHARACTER_CLASS),
    javaLowerCase javaUpperCase javaWhitespace javaMirrored javaLetter javaDigit javaLetterOrDigit
    javaAlphabetic, general categories (L Lu Ll Lt Lm Lo M Mn Mc Me N Nd Nl No P Pc Pd Ps Pe Pi Pf Po S Sm
    Sc Sk So Z Zs Zl Zp C Cc Cf Co Cn, also as IsL / gc=L / general_category=L), IsAlphabetic IsLetter
    IsDigit IsLowercase IsUppercase IsWhite_Space IsPunctuation IsControl IsIdeographic (binary
    properties); non-ASCII category tables come from the host's Unicode database (Python's unicodedata,
    a newer Unicode version than Java 8's: parity for code points assigned since then is unpinned);
  * groups: capturing, named (?<name>X) with \\k<name>, non-capturing (?:X), atomic (?>X), lookahead
    (?=X) (?!X), lookbehind (?<=X) (?<!X) with a bounded maximum length (as Java requires);
  * alternation; greedy, lazy and possessive quantifiers * + ? {n} {n,} {n,m};
  * anchors ^ $ \\b \\B \\A \\z \\Z \\G; backreferences \\1..\\9;
  * flags (?idmsuxU-idmsuxU) and (?flags:X), scoped like Java's: CASE_INSENSITIVE (US-ASCII, or with
    UNICODE_CASE the host's simple case mappings), MULTILINE, DOTALL, UNIX_LINES, COMMENTS,
    UNICODE_CHARACTER_CLASS (\\d \\w \\s and POSIX classes from Unicode properties).
Unsupported (CANON_EQ, a lookbehind without an obvious maximum length, more than 9 groups) raises
`RegexUnsupported`, which the analyzer reports as a failed metric — there is no CPU fallback.
"""
import struct
import sys
import unicodedata

# opcodes (deequ_amd/csrc/regex.hip)
OP_CHAR, OP_CLASS, OP_ANY, OP_SPLIT, OP_JMP, OP_SAVE, OP_ASSERT, OP_BACKREF, OP_LOOK, OP_LOOKEND, OP_MARK, \
    OP_CHECK, OP_MATCH, OP_ATOMIC, OP_ATOMIC_END, OP_STEPBACK, OP_ATPOS = range(1, 18)
A_BOL, A_EOL, A_WORDB, A_NWORDB, A_BEGIN, A_END, A_ENDZ, A_MBOL, A_MEOL, A_EOL_UNIX, A_MBOL_UNIX, A_MEOL_UNIX, \
    A_ENDZ_UNIX = range(13)
MAX_CP = 0x10FFFF
MAGIC = 0x52454758  # "REGX"

# java.util.regex.Pattern flags (inline letters)
F_UNIX_LINES, F_CASE_INSENSITIVE, F_COMMENTS, F_MULTILINE, F_DOTALL, F_UNICODE_CASE, F_UNICODE_CLASS = \
    1, 2, 4, 8, 32, 64, 256
FLAG_LETTERS = {"d": F_UNIX_LINES, "i": F_CASE_INSENSITIVE, "x": F_COMMENTS, "m": F_MULTILINE, "s": F_DOTALL,
                "u": F_UNICODE_CASE, "U": F_UNICODE_CLASS}


from .metrics import UnsupportedOnDevice


class RegexUnsupported(UnsupportedOnDevice):
    pass


# ---- parser -> AST --------------------------------------------------------------------------------
# nodes: ("char", cp) ("class", ranges) ("cat", [..]) ("alt", [..]) ("group", idx|None, node)
#        ("rep", node, min, max|None, greedy) ("assert", kind) ("backref", n, ci) ("look", neg, node)
#        ("lookbehind", neg, node, minlen, maxlen) ("atomic", node)

DIGIT = [(48, 57)]
SPACE = [(9, 13), (32, 32)]  # [ \t\n\x0B\f\r]
WORD = [(48, 57), (65, 90), (95, 95), (97, 122)]
LINE_TERMS = [(10, 10), (13, 13), (0x85, 0x85), (0x2028, 0x2029)]
HSPACE = [(9, 9), (32, 32), (0xA0, 0xA0), (0x1680, 0x1680), (0x180E, 0x180E), (0x2000, 0x200A), (0x202F, 0x202F),
          (0x205F, 0x205F), (0x3000, 0x3000)]
VSPACE = [(10, 13), (0x85, 0x85), (0x2028, 0x2029)]
ALL = [(0, MAX_CP)]

POSIX = {  # java.util.regex.Pattern's US-ASCII POSIX classes
    "Lower": [(97, 122)], "Upper": [(65, 90)], "ASCII": [(0, 127)], "Alpha": [(65, 90), (97, 122)],
    "Digit": [(48, 57)], "Alnum": [(48, 57), (65, 90), (97, 122)],
    "Punct": [(33, 47), (58, 64), (91, 96), (123, 126)], "Graph": [(33, 126)], "Print": [(32, 126)],
    "Blank": [(9, 9), (32, 32)], "Cntrl": [(0, 31), (127, 127)], "XDigit": [(48, 57), (65, 70), (97, 102)],
    "Space": [(9, 13), (32, 32)],
}


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


def _intersect(a, b):
    a, b = _normalize(a), _normalize(b)
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if lo <= hi:
            out.append((lo, hi))
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def _from_predicate(pred):
    """Code point ranges where pred(cp) holds, over the whole Unicode range (host Unicode database)."""
    out, start = [], None
    for cp in range(MAX_CP + 1):
        if pred(cp):
            if start is None:
                start = cp
        elif start is not None:
            out.append((start, cp - 1))
            start = None
    if start is not None:
        out.append((start, MAX_CP))
    return out


_CATEGORY_CACHE = {}


def _categories():
    """General category -> ranges, computed once from unicodedata (Unicode %s on this host)."""
    if not _CATEGORY_CACHE:
        runs = {}
        prev, start = None, 0
        for cp in range(MAX_CP + 2):
            cat = unicodedata.category(chr(cp)) if cp <= MAX_CP else None
            if cat != prev:
                if prev is not None:
                    runs.setdefault(prev, []).append((start, cp - 1))
                prev, start = cat, cp
        for cat, r in runs.items():
            _CATEGORY_CACHE[cat] = r
            _CATEGORY_CACHE.setdefault(cat[0], []).extend(r)
        for k in list(_CATEGORY_CACHE):
            _CATEGORY_CACHE[k] = _normalize(_CATEGORY_CACHE[k])
    return _CATEGORY_CACHE


def _cat(*names):
    c = _categories()
    out = []
    for n in names:
        out += c.get(n, [])
    return _normalize(out)


def _property(name, unicode_class):
    """Ranges of \\p{name} (java.util.regex.Pattern property names)."""
    raw = name
    if name in POSIX:
        if not unicode_class:
            return POSIX[name]
        uni = {"Lower": lambda: _cat("Ll"), "Upper": lambda: _cat("Lu"), "ASCII": lambda: POSIX["ASCII"],
               "Alpha": lambda: _cat("L", "Nl"), "Digit": lambda: _cat("Nd"), "Alnum": lambda: _cat("L", "Nl", "Nd"),
               "Punct": lambda: _cat("P"), "Graph": lambda: _negate(_cat("Zs", "Zl", "Zp", "Cc", "Cs", "Cn")),
               "Print": lambda: _normalize(_negate(_cat("Zs", "Zl", "Zp", "Cc", "Cs", "Cn")) + _cat("Zs")),
               "Blank": lambda: _normalize(_cat("Zs") + [(9, 9)]), "Cntrl": lambda: _cat("Cc"),
               "XDigit": lambda: _normalize(_cat("Nd") + [(48, 57), (65, 70), (97, 102)]),
               "Space": lambda: _normalize(_cat("Zs", "Zl", "Zp") + [(9, 13), (0x85, 0x85)])}
        return uni[name]()
    java = {"javaLowerCase": lambda: _cat("Ll"), "javaUpperCase": lambda: _cat("Lu"),
            "javaWhitespace": lambda: _normalize([(9, 13), (28, 31)] + _negate(_negate(_cat("Zs", "Zl", "Zp")) +
                                                                                [(0xA0, 0xA0), (0x2007, 0x2007),
                                                                                 (0x202F, 0x202F)])),
            "javaMirrored": lambda: _from_predicate(lambda c: unicodedata.mirrored(chr(c)) == 1),
            "javaLetter": lambda: _cat("L"), "javaDigit": lambda: _cat("Nd"),
            "javaLetterOrDigit": lambda: _cat("L", "Nd"), "javaAlphabetic": lambda: _cat("L", "Nl"),
            "javaSpaceChar": lambda: _cat("Zs", "Zl", "Zp"), "javaISOControl": lambda: [(0, 31), (127, 159)],
            "javaTitleCase": lambda: _cat("Lt"), "javaDefined": lambda: _negate(_cat("Cn"))}
    if name in java:
        return java[name]()
    for prefix in ("general_category=", "gc=", "Is"):
        if name.startswith(prefix):
            name = name[len(prefix):]
            break
    cats = _categories()
    if name in cats or name in ("L", "M", "N", "P", "S", "Z", "C"):
        return _cat(name)
    if name == "LC" or name == "L&":
        return _cat("Lu", "Ll", "Lt")
    binary = {"Alphabetic": lambda: _cat("L", "Nl"), "Letter": lambda: _cat("L"), "Digit": lambda: _cat("Nd"),
              "Lowercase": lambda: _cat("Ll"), "Uppercase": lambda: _cat("Lu"), "Titlecase": lambda: _cat("Lt"),
              "White_Space": lambda: _normalize(_cat("Zs", "Zl", "Zp") + [(9, 13), (0x85, 0x85)]),
              "WhiteSpace": lambda: _normalize(_cat("Zs", "Zl", "Zp") + [(9, 13), (0x85, 0x85)]),
              "Punctuation": lambda: _cat("P"), "Control": lambda: _cat("Cc"),
              "Ideographic": lambda: _from_predicate(lambda c: "CJK" in unicodedata.name(chr(c), "")
                                                      and unicodedata.category(chr(c)) in ("Lo", "Nl")),
              "Hex_Digit": lambda: [(48, 57), (65, 70), (97, 102), (0xFF10, 0xFF19), (0xFF21, 0xFF26),
                                    (0xFF41, 0xFF46)],
              "Assigned": lambda: _negate(_cat("Cn")), "Noncharacter_Code_Point":
                  lambda: _normalize([(0xFDD0, 0xFDEF)] + [(p * 0x10000 + 0xFFFE, p * 0x10000 + 0xFFFF)
                                                          for p in range(17)])}
    key = name.replace(" ", "_")
    for k, fn in binary.items():
        if k.lower() == key.lower():
            return fn()
    raise RegexUnsupported("unknown character property \\p{%s}" % raw)


def _case_closure(ranges, unicode_case):
    """The ranges plus every case variant of their code points: Java's CASE_INSENSITIVE compares
    US-ASCII letters only; with UNICODE_CASE, Character.toUpperCase / toLowerCase (here the host's simple case
    mappings)."""
    out = list(ranges)
    for lo, hi in ranges:
        for a, b, d in ((97, 122, -32), (65, 90, 32)):
            l2, h2 = max(lo, a), min(hi, b)
            if l2 <= h2:
                out.append((l2 + d, h2 + d))
        if unicode_case and hi >= 128:
            lo2 = max(lo, 128)
            if hi - lo2 > 0x30000:
                continue  # a (negated) class this wide already holds both cases of every letter it can
            for cp in range(lo2, hi + 1):
                ch = chr(cp)
                for v in (ch.upper(), ch.lower(), ch.title()):
                    if len(v) == 1 and v != ch:
                        out.append((ord(v), ord(v)))
                        for w in (v.upper(), v.lower()):  # e.g. Kelvin sign -> k -> K
                            if len(w) == 1:
                                out.append((ord(w), ord(w)))
    return _normalize(out)


class _Parser:
    def __init__(self, pattern, flags=0):
        self.p = pattern
        self.i = 0
        self.ngroups = 0
        self.names = {}
        self.flags = flags

    def peek(self, k=0):
        j = self.i + k
        return self.p[j] if j < len(self.p) else None

    def take(self):
        if self.i >= len(self.p):
            raise RegexUnsupported("unexpected end of pattern")
        c = self.p[self.i]
        self.i += 1
        return c

    def skip_comments(self):
        """COMMENTS: whitespace and '#' to end of line are ignored outside of escapes."""
        if not self.flags & F_COMMENTS:
            return
        while self.i < len(self.p):
            c = self.p[self.i]
            if c in " \t\n\x0b\f\r":
                self.i += 1
            elif c == "#":
                while self.i < len(self.p) and self.p[self.i] not in "\n\r\x85  ":
                    self.i += 1
            else:
                break

    def parse(self):
        node = self.alt()
        if self.i != len(self.p):
            raise RegexUnsupported("unbalanced ')' at %d" % self.i)
        return node

    def alt(self):
        saved = self.flags  # an inline (?f) lasts to the end of the enclosing group
        branches = [self.cat()]
        while self.peek() == "|":
            self.take()
            branches.append(self.cat())
        self.flags = saved
        return branches[0] if len(branches) == 1 else ("alt", branches)

    def cat(self):
        items = []
        while True:
            self.skip_comments()
            if self.peek() is None or self.peek() in "|)":
                break
            node = self.repeat()
            if node is not None:
                items.append(node)
        return ("cat", items)

    def repeat(self):
        atom = self.atom()
        if atom is None:  # a bare flag group (?i) or an empty \Q\E
            return None
        while True:
            self.skip_comments()
            c = self.peek()
            if c in ("*", "+", "?"):
                self.take()
                lo, hi = {"*": (0, None), "+": (1, None), "?": (0, 1)}[c]
            elif c == "{" and self._is_counted():
                lo, hi = self._counted()
            else:
                return atom
            kind = "greedy"
            if self.peek() == "?":
                self.take()
                kind = "lazy"
            elif self.peek() == "+":
                self.take()
                kind = "possessive"
            if hi is not None and hi < lo:
                raise RegexUnsupported("illegal repetition range {%d,%d}" % (lo, hi))
            if atom[0] in ("assert", "look", "lookbehind") and lo <= 1:
                # Java accepts X? / X* / X{0,1} on a zero-width assertion: it then matches with or without it
                atom = ("cat", []) if lo == 0 else atom
                continue
            node = ("rep", atom, lo, hi, kind != "lazy")
            atom = ("atomic", node) if kind == "possessive" else node

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

    def _flag_group(self):
        """(?idmsuxU-idmsuxU) or (?idmsuxU-idmsuxU:X); the '(?' is consumed."""
        on, off, neg = 0, 0, False
        while True:
            c = self.take()
            if c == "-":
                neg = True
            elif c in FLAG_LETTERS:
                if neg:
                    off |= FLAG_LETTERS[c]
                else:
                    on |= FLAG_LETTERS[c]
            elif c == "c":
                raise RegexUnsupported("CANON_EQ is not supported")
            elif c == ")":
                self.flags = (self.flags | on) & ~off
                return None
            elif c == ":":
                saved = self.flags
                self.flags = (self.flags | on) & ~off
                node = ("group", None, self.alt())
                self.flags = saved
                self._close()
                return node
            else:
                raise RegexUnsupported("unknown inline modifier %r" % c)

    def _close(self):
        if self.peek() != ")":
            raise RegexUnsupported("missing ')'")
        self.take()

    def _char_node(self, cp):
        if self.flags & F_CASE_INSENSITIVE:
            r = _case_closure([(cp, cp)], self.flags & F_UNICODE_CASE)
            if r != [(cp, cp)]:
                return ("class", r)
        return ("char", cp)

    def atom(self):
        c = self.take()
        if c == "(":
            if self.peek() == "?":
                self.take()
                k = self.peek()
                if k == ":":
                    self.take()
                    node = ("group", None, self.alt())
                elif k in ("=", "!"):
                    self.take()
                    node = ("look", k == "!", self.alt())
                elif k == ">":
                    self.take()
                    node = ("atomic", ("group", None, self.alt()))
                elif k == "<" and self.peek(1) in ("=", "!"):
                    self.take()
                    neg = self.take() == "!"
                    body = self.alt()
                    lo, hi = _length_bounds(body)
                    if hi is None:
                        raise RegexUnsupported("Look-behind group does not have an obvious maximum length")
                    node = ("lookbehind", neg, body, lo, hi)
                elif k == "<":
                    self.take()
                    name = ""
                    while self.peek() not in (">", None):
                        name += self.take()
                    self.take()
                    if not name or not (name[0].isascii() and name[0].isalpha()) or \
                            not all(ch.isascii() and ch.isalnum() for ch in name):
                        raise RegexUnsupported("capturing group name %r" % name)
                    if name in self.names:
                        raise RegexUnsupported("named capturing group <%s> is already defined" % name)
                    self.ngroups += 1
                    idx = self.ngroups
                    self.names[name] = idx
                    node = ("group", idx, self.alt())
                else:
                    return self._flag_group()
            else:
                self.ngroups += 1
                idx = self.ngroups
                node = ("group", idx, self.alt())
            self._close()
            return node
        if c == "[":
            return ("class", self._class())
        if c == ".":
            if self.flags & F_DOTALL:
                return ("class", ALL)
            return ("class", _negate([(10, 10)] if self.flags & F_UNIX_LINES else LINE_TERMS))
        if c == "^":
            if self.flags & F_MULTILINE:
                return ("assert", A_MBOL_UNIX if self.flags & F_UNIX_LINES else A_MBOL)
            return ("assert", A_BOL)
        if c == "$":
            if self.flags & F_MULTILINE:
                return ("assert", A_MEOL_UNIX if self.flags & F_UNIX_LINES else A_MEOL)
            return ("assert", A_EOL_UNIX if self.flags & F_UNIX_LINES else A_EOL)
        if c == "\\":
            return self._escape(in_class=False)
        if c in ")*+?{":
            raise RegexUnsupported("dangling metacharacter %r" % c)  # Java: "Dangling meta character" / "Illegal repetition"
        return self._char_node(ord(c))

    def _predef(self, ranges):
        return ("class", ranges)

    def _escape(self, in_class):
        c = self.take()
        uc = self.flags & F_UNICODE_CLASS
        simple = {"t": 9, "n": 10, "r": 13, "f": 12, "e": 27, "a": 7}
        if c in simple:
            return self._char_node(simple[c]) if not in_class else ("char", simple[c])
        if c == "x":
            if self.peek() == "{":
                self.take()
                h = ""
                while self.peek() != "}":
                    h += self.take()
                self.take()
                cp = int(h, 16)
                if cp > MAX_CP:
                    raise RegexUnsupported("hexadecimal codepoint is too big")
            else:
                cp = int(self.take() + self.take(), 16)
            return self._char_node(cp) if not in_class else ("char", cp)
        if c == "u":
            cp = int("".join(self.take() for _ in range(4)), 16)
            if 0xD800 <= cp <= 0xDBFF and self.p[self.i:self.i + 2] == "\\u":  # a surrogate pair
                lo = int(self.p[self.i + 2:self.i + 6], 16)
                if 0xDC00 <= lo <= 0xDFFF:
                    self.i += 6
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00)
            return self._char_node(cp) if not in_class else ("char", cp)
        if c == "0":
            o = ""
            while len(o) < 3 and self.peek() is not None and self.peek() in "01234567":
                if len(o) == 2 and int(o + self.peek(), 8) > 0o377:
                    break
                o += self.take()
            if not o:
                raise RegexUnsupported("illegal octal escape sequence")
            return self._char_node(int(o, 8)) if not in_class else ("char", int(o, 8))
        if c == "c":
            cp = ord(self.take()) ^ 64
            return self._char_node(cp) if not in_class else ("char", cp)
        if c == "d":
            return self._predef(_cat("Nd") if uc else DIGIT)
        if c == "D":
            return self._predef(_negate(_cat("Nd") if uc else DIGIT))
        if c == "s":
            return self._predef(_property("White_Space", True) if uc else SPACE)
        if c == "S":
            return self._predef(_negate(_property("White_Space", True) if uc else SPACE))
        if c == "w":
            return self._predef(_unicode_word() if uc else WORD)
        if c == "W":
            return self._predef(_negate(_unicode_word() if uc else WORD))
        if c == "h":
            return self._predef(HSPACE)
        if c == "H":
            return self._predef(_negate(HSPACE))
        if c == "v":
            return self._predef(VSPACE)
        if c == "V":
            return self._predef(_negate(VSPACE))
        if c in "pP":
            if self.peek() == "{":
                self.take()
                name = ""
                while self.peek() not in ("}", None):
                    name += self.take()
                self.take()
            else:
                name = self.take()
            neg = c == "P"
            if name.startswith("^"):
                neg, name = not neg, name[1:]
            r = _property(name, uc)
            if self.flags & F_CASE_INSENSITIVE and name in ("Lower", "Upper", "javaLowerCase", "javaUpperCase",
                                                            "Ll", "Lu", "Lt", "IsLowercase", "IsUppercase"):
                r = _case_closure(r, True)
            return ("class", _negate(r) if neg else r)
        if c == "Q":
            end = self.p.find("\\E", self.i)
            lit = self.p[self.i:] if end < 0 else self.p[self.i:end]
            self.i = len(self.p) if end < 0 else end + 2
            if in_class:
                return ("quoted", [ord(ch) for ch in lit])
            nodes = [self._char_node(ord(ch)) for ch in lit]
            return ("cat", nodes) if nodes else None
        if not in_class:
            if c == "b":
                return ("assert", A_WORDB)
            if c == "B":
                return ("assert", A_NWORDB)
            if c == "A":
                return ("assert", A_BEGIN)
            if c == "G":  # end of the previous match: the first find() starts at 0
                return ("assert", A_BEGIN)
            if c == "z":
                return ("assert", A_END)
            if c == "Z":
                return ("assert", A_ENDZ_UNIX if self.flags & F_UNIX_LINES else A_ENDZ)
            if c == "R":  # Java 8: (?:\u000D\u000A|[\u000A\u000B\u000C\u000D\u0085  ])
                return ("atomic", ("alt", [("cat", [("char", 13), ("char", 10)]), ("class", VSPACE)]))
            if c == "k":
                if self.take() != "<":
                    raise RegexUnsupported("\\k is not followed by '<' for named capturing group")
                name = ""
                while self.peek() not in (">", None):
                    name += self.take()
                self.take()
                if name not in self.names:
                    raise RegexUnsupported("named capturing group <%s> does not exist" % name)
                return ("backref", self.names[name], self._backref_ci())
            if c.isdigit() and c != "0":
                # Java: a multi-digit reference is taken while the group exists
                n = int(c)
                while self.peek() is not None and self.peek().isdigit() and int(str(n) + self.peek()) <= self.ngroups:
                    n = int(str(n) + self.take())
                return ("backref", n, self._backref_ci())
        if c.isalpha() or c.isdigit():
            raise RegexUnsupported("illegal/unsupported escape sequence \\%s" % c)
        return self._char_node(ord(c)) if not in_class else ("char", ord(c))

    def _backref_ci(self):
        if not self.flags & F_CASE_INSENSITIVE:
            return 0
        return 2 if self.flags & F_UNICODE_CASE else 1

    def _class(self):
        """A character class after '[': union of its items, '&&' intersections, nested classes."""
        neg = False
        if self.peek() == "^":
            self.take()
            neg = True
        acc = None  # result of the intersections so far
        ranges = []
        first = True
        while True:
            if self.flags & F_COMMENTS:
                self.skip_comments()
            c = self.peek()
            if c is None:
                raise RegexUnsupported("unclosed character class")
            if c == "]" and not first:
                self.take()
                break
            first = False
            if c == "[":
                self.take()
                ranges.extend(self._class())
                continue
            if c == "&" and self.peek(1) == "&":
                self.i += 2
                acc = ranges if acc is None else _intersect(acc, ranges)
                ranges = []
                continue
            lo = self._class_atom()
            if lo[0] == "class":
                ranges.extend(lo[1])
                continue
            if lo[0] == "quoted":
                ranges.extend((cp, cp) for cp in lo[1])
                continue
            lo = lo[1]
            if self.peek() == "-" and self.peek(1) not in (None, "]", "[") and \
                    not (self.peek(1) == "&" and self.peek(2) == "&"):
                self.take()
                hi = self._class_atom()
                if hi[0] != "char":
                    raise RegexUnsupported("illegal character range")
                if hi[1] < lo:
                    raise RegexUnsupported("illegal character range")
                ranges.append((lo, hi[1]))
            else:
                ranges.append((lo, lo))
        if acc is not None:
            ranges = _intersect(acc, ranges) if ranges else acc
        ranges = _normalize(ranges)
        if self.flags & F_CASE_INSENSITIVE:
            ranges = _case_closure(ranges, self.flags & F_UNICODE_CASE)
        return _negate(ranges) if neg else ranges

    def _class_atom(self):
        c = self.take()
        if c == "\\":
            return self._escape(in_class=True)
        return ("char", ord(c))


def _unicode_word():
    # UNICODE_CHARACTER_CLASS \w: [\p{Alpha}\p{gc=Mn}\p{gc=Me}\p{gc=Mc}\p{Digit}\p{gc=Pc}\p{IsJoin_Control}]
    return _normalize(_cat("L", "Nl", "Mn", "Me", "Mc", "Nd", "Pc") + [(0x200C, 0x200D)])


def _length_bounds(n):
    """(min, max) length in code points of what node n matches; max None when unbounded."""
    k = n[0]
    if k in ("char", "class"):
        return 1, 1
    if k in ("assert", "look", "lookbehind"):
        return 0, 0
    if k == "backref":
        return 0, None
    if k == "cat":
        lo, hi = 0, 0
        for x in n[1]:
            a, b = _length_bounds(x)
            lo += a
            hi = None if hi is None or b is None else hi + b
        return lo, hi
    if k == "alt":
        bs = [_length_bounds(x) for x in n[1]]
        return min(b[0] for b in bs), (None if any(b[1] is None for b in bs) else max(b[1] for b in bs))
    if k == "group":
        return _length_bounds(n[2])
    if k == "atomic":
        return _length_bounds(n[1])
    if k == "rep":
        a, b = _length_bounds(n[1])
        hi = None if n[3] is None or b is None else b * n[3]
        return a * n[2], hi
    return 0, None


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
            self.emit(OP_BACKREF, n[1], n[2])
        elif k == "look":
            look = self.emit(OP_LOOK, 0, 1 if n[1] else 0)
            self.gen(n[2])
            self.emit(OP_LOOKEND)
            self.code[look][1] = len(self.code)
        elif k == "lookbehind":
            # LOOK (frame at the current position p), STEPBACK tries start positions p - k for k = min..max code
            # points (Java's Behind node order), the body must end exactly at p (ATPOS), LOOKEND as for lookahead
            _, neg, body, lo, hi = n
            look = self.emit(OP_LOOK, 0, 1 if neg else 0)
            self.emit(OP_STEPBACK, lo, hi)
            self.gen(body)
            self.emit(OP_ATPOS)
            self.emit(OP_LOOKEND)
            self.code[look][1] = len(self.code)
        elif k == "atomic":
            # (?>X): once X matched, its untried alternatives are dropped (ATOMIC_END cuts the branch frames above
            # the ATOMIC marker, keeping the capture / loop undo records)
            self.emit(OP_ATOMIC)
            self.gen(n[1])
            self.emit(OP_ATOMIC_END)
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
    if k in ("char", "class", "backref"):
        return k == "backref"
    if k in ("assert", "look", "lookbehind"):
        return True
    if k == "atomic":
        return _nullable(n[1])
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


def compile_regex(pattern, flags=0):
    """Pattern.compile(pattern, flags).  `flags` are java.util.regex.Pattern's flag bits (F_*)."""
    p = _Parser(pattern, flags)
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
