"""A small reader for the literal Rust expressions the reference's unit tests are
written in (test infrastructure for make_rule_kats.py; it reads reference test
sources as text and never executes them).

parse_expr() turns an expression such as
    FdoTeamState::NoWedding { re_players: FdoPlayerSet::from_vec(vec![FdoPlayer::TOP]) }
into nested tuples:
    ("path", "A::B")              a path / enum variant / variable name
    ("call", "A::b", [args])      a call of a path (also Some(x), macros like vec![...])
    ("struct", "A::B", {f: v})    a struct literal
    ("list", [items])             [a, b] and vec![a, b]
    ("method", obj, "m", [args])  obj.m(args)
    ("ref", expr) / ("not", expr) / ("neg", expr)
    ("tuple", [items])            (a, b)
    int / bool / str
"""
import re

TOKEN = re.compile(r"""
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<num>\d+(?:\.\d+)?(?:_?[uif](?:8|16|32|64|size))?)
  | (?P<str>"(?:\\.|[^"\\])*")
  | (?P<char>'(?:\\.|[^'\\])')
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:::[A-Za-z_][A-Za-z0-9_]*)*(?:::<[^>]*>)?)
  | (?P<op>==|!=|<=|>=|&&|\|\||::|->|=>|[()\[\]{},;:&!=.<>+\-*/|?#])
""", re.X | re.S)


def tokenize(src):
    out = []
    pos = 0
    while pos < len(src):
        m = TOKEN.match(src, pos)
        if not m:
            raise ValueError("cannot tokenize at %r" % src[pos:pos + 40])
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        out.append((kind, m.group()))
    return out


class Parser:
    def __init__(self, tokens):
        self.t = tokens
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self, val=None):
        tok = self.t[self.i]
        if val is not None and tok[1] != val:
            raise ValueError("expected %r got %r at %d" % (val, tok, self.i))
        self.i += 1
        return tok

    def at(self, val):
        return self.peek()[1] == val

    def items(self, close):
        xs = []
        while not self.at(close):
            xs.append(self.expr())
            if self.at(","):
                self.take(",")
        self.take(close)
        return xs

    def expr(self):
        e = self.unary()
        while self.at("==") or self.at("!="):
            op = self.take()[1]
            e = ("cmp", op, e, self.unary())
        while self.at("&&"):
            self.take()
            e = ("and", e, self.unary())
        return e

    def unary(self):
        if self.at("&"):
            self.take()
            if self.peek()[1] == "mut":
                self.take()
            return ("ref", self.unary())
        if self.at("!"):
            self.take()
            return ("not", self.unary())
        if self.at("-"):
            self.take()
            v = self.unary()
            return -v if isinstance(v, int) else ("neg", v)
        return self.postfix(self.primary())

    def postfix(self, e):
        while True:
            if self.at("."):
                self.take()
                kind, name = self.take()
                if kind == "num":       # tuple field .0
                    e = ("field", e, int(name))
                    continue
                args = []
                if self.at("("):
                    self.take("(")
                    args = self.items(")")
                    e = ("method", e, name, args)
                else:
                    e = ("field", e, name)
            elif self.at("?"):
                self.take()
            elif self.at("["):
                self.take()
                idx = self.expr()
                self.take("]")
                e = ("index", e, idx)
            else:
                return e

    def primary(self):
        kind, val = self.peek()
        if kind == "num":
            self.take()
            v = re.match(r"\d+(?:\.\d+)?", val).group()
            return float(v) if "." in v else int(v)
        if kind == "str":
            self.take()
            return val[1:-1]
        if kind == "char":
            self.take()
            return val[1:-1]
        if val == "(":
            self.take()
            xs = self.items(")")
            return xs[0] if len(xs) == 1 else ("tuple", xs)
        if val == "[":
            self.take()
            # [x; n] repetition
            first = self.expr() if not self.at("]") else None
            if first is not None and self.at(";"):
                self.take()
                n = self.expr()
                self.take("]")
                return ("list", [first] * n)
            xs = [] if first is None else [first]
            if self.at(","):
                self.take(",")
            xs += self.items("]")
            return ("list", xs)
        if kind == "ident":
            self.take()
            name = re.sub(r"::<[^>]*>$", "", val)
            if name in ("true", "false"):
                return name == "true"
            if self.at("!"):              # macro
                self.take()
                opener = self.take()[1]
                close = {"(": ")", "[": "]", "{": "}"}[opener]
                args = self.items(close)
                return ("list", args) if name == "vec" else ("call", name + "!", args)
            if self.at("("):
                self.take()
                return ("call", name, self.items(")"))
            if self.at("{") and name[:1].isupper():
                self.take()
                fields = {}
                while not self.at("}"):
                    fname = self.take()[1]
                    if self.at(":"):
                        self.take(":")
                        fields[fname] = self.expr()
                    else:
                        fields[fname] = ("path", fname)
                    if self.at(","):
                        self.take(",")
                self.take("}")
                return ("struct", name, fields)
            return ("path", name)
        raise ValueError("unexpected token %r" % (self.peek(),))


def parse_expr(src):
    p = Parser(tokenize(src))
    e = p.expr()
    return e


def balanced(text, start, open_ch="(", close_ch=")"):
    """Index just past the bracket matching text[start] == open_ch (strings and comments aware)."""
    depth = 0
    i = start
    while i < len(text):
        c = text[i]
        if text.startswith("//", i):
            i = text.index("\n", i)
            continue
        if c == '"':
            j = i + 1
            while text[j] != '"':
                j += 2 if text[j] == "\\" else 1
            i = j + 1
            continue
        if c == open_ch:
            depth += 1
        elif c == close_ch:
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1
    raise ValueError("unbalanced")


def test_functions(text):
    """(name, body) of every `#[test] fn name() { body }` in a source file."""
    out = []
    for m in re.finditer(r"#\[test\]\s*(?:pub\s+)?fn\s+(\w+)\s*\(\)\s*\{", text):
        start = m.end() - 1
        end = balanced(text, start, "{", "}")
        out.append((m.group(1), text[start + 1:end - 1]))
    return out


def statements(body):
    """Split a function body into top-level statements (ending at ';' or a closing block)."""
    toks = tokenize(body)
    out, cur, depth = [], [], 0
    for tok in toks:
        cur.append(tok)
        if tok[1] in "([{":
            depth += 1
        elif tok[1] in ")]}":
            depth -= 1
            if depth == 0 and tok[1] == "}" and len(cur) > 1 and cur[0][1] in ("match", "if", "for", "loop"):
                out.append(cur)
                cur = []
        elif tok[1] == ";" and depth == 0:
            out.append(cur[:-1])
            cur = []
    if cur:
        out.append(cur)
    return out


def parse_tokens(tokens):
    return Parser(tokens).expr()
