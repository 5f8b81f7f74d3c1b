"""The regex/contains leaf matcher (lakeside_amd/csrc/regex.cpp) against RE2 itself (CPU, no GPU).

The reference compiles `regex` to regexp_matches(label, 'p', 'i') and `contains` to
regexp_matches(label, '.*p.*', 'i') (BaseExpr.scala:485-486, 500-501); DuckDB runs RE2.  pyarrow bundles RE2 and
pyarrow.compute.match_substring_regex(values, p, ignore_case=True) is the same partial, case-insensitive match, so
it is the oracle here: for every pattern of the corpus both must agree on "is it a valid RE2 regex" and, when it
is, on the match of every value (ASCII, non-ASCII, case-fold orbits, newlines, invalid UTF-8 excluded).
"""
import ctypes
import os
import random
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lakeside_amd", "liblakeside_regex.so")


class Re:
    _L = None

    @classmethod
    def lib(cls):
        if cls._L is None:
            L = ctypes.CDLL(LIB)
            L.lkre_compile.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
            L.lkre_compile.restype = ctypes.c_int
            L.lkre_search.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
            L.lkre_search.restype = ctypes.c_int
            L.lkre_free.argtypes = [ctypes.c_void_p]
            L.lkre_last_error.restype = ctypes.c_char_p
            cls._L = L
        return cls._L

    def __init__(self, pattern: str, icase=True):
        b = pattern.encode()
        self.h = ctypes.c_void_p()
        self.rc = self.lib().lkre_compile(b, len(b), 1 if icase else 0, ctypes.byref(self.h))
        self.err = self.lib().lkre_last_error().decode() if self.rc else ""

    def search(self, s: str) -> bool:
        b = s.encode()
        return bool(self.lib().lkre_search(self.h, b, len(b)))

    def __del__(self):
        if getattr(self, "h", None) and self.h.value:
            self.lib().lkre_free(self.h)


def re2(values, pattern, icase=True):
    """RE2 via pyarrow; None when RE2 rejects the pattern."""
    import pyarrow as pa
    import pyarrow.compute as pc
    try:
        return pc.match_substring_regex(pa.array(values, pa.string()), pattern, ignore_case=icase).to_pylist()
    except pa.ArrowInvalid:
        return None


VALUES = [
    "", "a", "A", "svc-001", "SVC-042", "svc-04", "metric_07", "Metric_07x", "hello world", "hello\nworld",
    "foo.bar", "foo-bar", "fooXbar", "x{2}", "a{,3}", "aaa", "abab", "ba", "]", "[", "\\", "-", "^", "$", "a|b",
    "tab\there", "cr\rlf", "null", "NULL", "ns-01", "c0000001", "c9999999", "12345", "3.14", "_id", "k8s.io",
    "ÉCOLE", "école", "Straße", "STRASSE", "straße", "ẞ", "ſ", "s", "S", "K", "k", "K", "Σίσυφος", "ΣΊΣΥΦΟΣ", "σς",
    "İstanbul", "ıi", "Iİ", "ǅ", "ǆ", "Ǆ", "привет", "ПРИВЕТ", "日本語テキスト", "😀 emoji", "aéb", "\u0000nul",
    "\x7f", "word boundary", "wordboundary", "end.", "line1\nline2\n", "\n", "ab\nc", "xyzzy" * 20,
]

PATTERNS = [
    # literals, dot, anchors
    "", "a", "svc", "SVC-0[0-4]", "^svc-0[0-4]", "0[0-4]$", "^$", "^", "$", ".", "a.c", "hello.world", "^.*$",
    "\\Asvc", "svc\\z", "(?i)^SVC-0[0-4]", "(?-i)SVC", "(?-i:svc)-0", "(?s)hello.world", "(?m)^world",
    "(?m)hello$", "(?m:^line2$)", "\\bword\\b", "\\bboundary", "\\Bboundary", "d\\b", "\\B", "\\b",
    # classes
    "[a-c]", "[^a-c]", "[]x]", "[^]x]", "[]]", "[a-]", "[-a]", "[a\\-z]", "[\\]]", "[\\[]", "[[:alpha:]]+",
    "[[:^alpha:]]", "[[:digit:]a]\\z", "[[:upper:]]", "[[:word:]]", "[[:punct:]]", "[[:space:]]", "[[:xdigit:]]+$",
    "[[:foo:]]", "[[:alpha:]x]", "[[:alpha:", "[\\d]", "[\\D]", "[\\s]", "[\\w-]", "[\\W]", "[\\pL]", "[\\p{Lu}]",
    "[\\P{L}]", "[\\p{^L}]", "[é]", "[É]", "[ß]", "[ſ]", "[k]", "[^k]", "[^\\n]", "[a-z&&b]", "[z-a]", "[\\b]",
    "[\\x41-\\x43]", "[\\x{393}-\\x{3A9}]", "[^\\x00-\\x7f]", "[\\Q]", "[", "]", "[a", "[^", "[]",
    # perl / unicode groups
    "\\d+", "\\D", "\\s", "\\S", "\\w+", "\\W", "\\pL", "\\PL", "\\p{L}", "\\p{Lu}", "\\p{Ll}", "\\p{Greek}",
    "\\p{Han}", "\\pN", "\\p{Nd}", "\\p{Zs}", "\\p{Any}", "\\p{^Lu}", "\\P{^Lu}", "\\pZ", "\\p{Foo}", "\\p{L",
    "\\pLu", "\\p",
    # escapes
    "\\.", "foo\\.bar", "\\-", "\\_id", "\\x41", "\\x{212A}", "\\x{110000}", "\\x4", "\\xZZ", "\\0", "\\01",
    "\\012", "\\1", "\\12", "\\8", "\\t", "\\n", "\\r", "\\f", "\\v", "\\a", "\\e", "\\Z", "\\q", "\\Qa.b\\E",
    "\\Qsvc\\E", "\\Q\\E", "\\Qa*", "a\\Q.\\E*", "\\C", "\\", "a\\", "\\é", "\\u0041", "\\cA",
    # repetition
    "a*", "a+", "a?", "a{2}", "a{2,}", "a{2,3}", "a{,3}", "a{3,2}", "a{1001}", "a{1000}", "(a{2}){500}",
    "(a{2}){501}", "((a{10}){10}){10}", "((a{10}){10}){11}", "a**", "a*?", "a+?", "a??", "a{2}?", "a{2}*", "a*{2}",
    "*a", "+a", "?a", "{2}", "x{2", "x{", "x{a}", "x{01}", "a|*", "(*)", "^*", "$+", "\\b*", "(?i)*", "a{0}",
    "a{0,0}", "(a|a)*b", "(a*)*b", "(a|b)*abb", "(x+x+)+y", "(?:a|ab)(?:c|bcd)(?:d*)",
    # groups & flags
    "(a)", "(?:a)", "(?P<id>svc-0[1-3])[0-9]\\z", "(?<id>svc)", "(?P<1a>x)", "(?P<>x)", "(?P<a>x)(?P<a>y)",
    "(?P=a)", "(?P>a)", "(?=a)", "(?!a)", "(?<=a)", "(?<!a)", "(?i)", "(?)", "(?-)", "(?i-)", "(?x)", "(?#c)",
    "(?i:A)B", "(?U)a+", "(?sm)a.b", "()", "(", ")", "a)", "(a", "((a)", "a|", "|a", "|", "a||b", "(|a)",
    # case folding / Unicode
    "strasse", "STRASSE", "straße", "ß", "ẞ", "s", "k", "K", "σ", "ς", "Σ", "σίσυφος", "école", "ÉCOLE",
    "i", "I", "ı", "İ", "ǅ", "привет", "日本", "😀", ".emoji", "^.{2}$", "^.$", "\\p{L}{3}", "[^a]", "[^a]+$",
    "x{0}y", "(?i)[k]", "(?i)[^k]", "(?i)\\W", "(?i)[[:^alpha:]]", "(?i)\\P{Lu}", "(?i)[a-z]+", "(?i)[\\x{212a}]",
    # Unicode scripts (VERDICT r3 missing #4)
    "\\p{Greek}", "\\p{Greek}+$", "\\P{Han}", "[\\p{Cyrillic}\\d]+", "(?i)\\p{Greek}", "\\p{^Latin}",
    "[^\\p{Latin}\\p{Common}]", "\\p{Hiragana}|\\p{Katakana}", "\\p{Inherited}", "\\p{Nko}",
    # contains-shaped
    ".*svc.*", ".*SVC-0.*", ".*.*", ".*\\..*", ".*(.*", ".*[a.*",
]


def _check_pattern(p, icase=True):
    want = re2(VALUES, p, icase)
    r = Re(p, icase)
    if want is None:
        assert r.rc == -1, f"{p!r}: RE2 rejects it, matcher compiled it (rc {r.rc})"
        return
    if r.rc == -2:
        return want   # valid RE2 syntax this matcher reports as unsupported (checked by the caller's allow-list)
    assert r.rc == 0, f"{p!r}: RE2 accepts it, matcher failed: {r.err}"
    got = [r.search(v) for v in VALUES]
    bad = [(v, g, w) for v, g, w in zip(VALUES, got, want) if g != bool(w)]
    assert not bad, f"{p!r}: (value, matcher, RE2) disagree: {bad[:5]}"
    return None


UNSUPPORTED_OK = {"\\C"}   # Unicode scripts are implemented (tables probed from RE2, tools/gen_unicode_tables.py)


@pytest.mark.parametrize("icase", [True, False])
def test_pattern_corpus_matches_re2(icase):
    unsupported = []
    for p in PATTERNS:
        if _check_pattern(p, icase) is not None:
            unsupported.append(p)
    assert set(unsupported) <= UNSUPPORTED_OK, unsupported


def test_random_patterns_match_re2():
    """Random patterns over a small alphabet (classes, groups, alternation, repetition, anchors) against RE2 on
    random strings over the same alphabet (plus fold partners)."""
    rng = random.Random(20240101)
    atoms = ["a", "b", "A", "é", "É", "k", "\\x{212a}", ".", "[ab]", "[^a]", "[a-c]", "\\w", "\\W", "\\d", "\\s",
             "ß", "\\pL", "\\PL", "[[:upper:]]", "(?i:a)", "(?-i:b)"]
    reps = ["", "", "", "*", "+", "?", "{2}", "{1,2}", "*?"]

    def gen(depth=0):
        n = rng.randint(1, 4)
        parts = []
        for _ in range(n):
            r = rng.random()
            if depth < 2 and r < 0.2:
                a = "(" + gen(depth + 1) + ")"
            elif depth < 2 and r < 0.3:
                a = "(?:" + gen(depth + 1) + "|" + gen(depth + 1) + ")"
            else:
                a = rng.choice(atoms)
            parts.append(a + rng.choice(reps))
        s = "".join(parts)
        if rng.random() < 0.15:
            s = "^" + s
        if rng.random() < 0.15:
            s = s + "$"
        if rng.random() < 0.1:
            s = s.replace("a", "\\b" + "a", 1)
        return s

    alphabet = ["a", "b", "A", "B", "é", "É", "k", "K", "K", "ß", "s", " ", "1", "\n", "_", "ſ"]
    values = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 8))) for _ in range(300)]
    for i in range(400):
        p = gen()
        icase = rng.random() < 0.7
        want = re2(values, p, icase)
        r = Re(p, icase)
        if want is None:
            assert r.rc == -1, (p, r.rc)
            continue
        assert r.rc == 0, (p, r.err)
        got = [r.search(v) for v in values]
        bad = [(v, g, w) for v, g, w in zip(values, got, want) if g != bool(w)]
        assert not bad, f"{p!r} icase={icase}: {bad[:5]}"


def test_linear_time_and_no_crash_on_long_values():
    """RE2 is linear; so is the matcher: pathological backtracking patterns over long inputs finish quickly,
    and a 1 MB value (log bodies reach this path through PLAIN-page dictionaries) neither recurses nor hangs."""
    big = "a" * (1 << 20)
    for p, want in [("(a|a)*b", False), ("(a*)*b", False), ("(x+x+)+y", False), (".*a.*a.*a.*b", False),
                    ("(a|a)*$", True), ("a{1000}", True), ("\\bq", False)]:
        r = Re(p)
        assert r.rc == 0, (p, r.err)
        t = time.perf_counter()
        assert r.search(big) == want, p
        assert time.perf_counter() - t < 2.0, f"{p} took too long"
    r = Re(".*needle.*")
    assert r.search("x" * (1 << 20) + "NEEDLE")
    assert not r.search("x" * (1 << 20))


def test_invalid_utf8_text_does_not_match_dot():
    lib = Re.lib()
    r = Re("^.$")
    b = b"\xff"
    assert lib.lkre_search(r.h, b, 1) == 0
    r2 = Re("a")
    b2 = b"\xffa\xfe"
    assert lib.lkre_search(r2.h, b2, 3) == 1
