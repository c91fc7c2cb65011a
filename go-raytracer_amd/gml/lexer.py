"""GML lexer + preprocessor (host front end).

Restates internal/gml/lexer.go: tokens (:17-65), identifiers/binders, numbers
(:396-423), strings with escapes (:429-463), `%` line comments, `/* */`
block comments, and the #include / #ifndef / #define / #endif subset
(:271-386) with include-cycle detection, resolved relative to the including
file.
"""
import os

EOF, ILLEGAL, ERROR, IDENT, BINDER, BOOLEAN, INT, FLOAT, STRING, LCURLY, RCURLY, LBRACKET, RBRACKET = range(13)
NAMES = ["EOF", "Illegal", "Error", "Ident", "Binder", "Boolean", "Integer", "Float", "String",
         "LCurly", "RCurly", "LBracket", "RBracket"]


class Token:
    __slots__ = ("type", "literal", "line", "col")

    def __init__(self, type_, literal, line, col):
        self.type = type_
        self.literal = literal
        self.line = line
        self.col = col

    def __repr__(self):
        return "Token(%s, %r, %d:%d)" % (NAMES[self.type], self.literal, self.line, self.col)


def _is_letter(c):
    return ("a" <= c <= "z") or ("A" <= c <= "Z")


def _is_digit(c):
    return "0" <= c <= "9"


class _Frame:
    __slots__ = ("input", "pos", "read_pos", "ch", "line", "col", "file")

    def __init__(self, text, file=""):
        self.input = text
        self.pos = 0
        self.read_pos = 0
        self.ch = ""
        self.line = 1
        self.col = 0
        self.file = file


class Lexer:
    def __init__(self, text, file=""):
        self.f = _Frame(text, file)
        self.stack = []
        self.active = {file} if file else set()
        self.defined = set()
        self.cond_depth = 0
        self._read()

    @classmethod
    def from_file(cls, path):
        path = os.path.abspath(path)
        with open(path, "r") as fh:
            return cls(fh.read(), path)

    # -- character reading (lexer.go readChar/popFrame) --
    def _read(self):
        f = self.f
        if f.ch == "\n":
            f.line += 1
            f.col = 1
        else:
            f.col += 1
        if f.read_pos >= len(f.input) and self.stack:
            self.active.discard(f.file)
            self.f = self.stack.pop()
            return
        if f.read_pos >= len(f.input):
            f.ch = ""
        else:
            f.ch = f.input[f.read_pos]
        f.pos = f.read_pos
        f.read_pos += 1

    def _peek(self):
        f = self.f
        return f.input[f.read_pos] if f.read_pos < len(f.input) else ""

    def _single(self, typ, line, col):
        t = Token(typ, self.f.ch, line, col)
        self._read()
        return t

    def next_token(self):
        while self.f.ch in (" ", "\t", "\n", "\r"):
            self._read()
        line, col = self.f.line, self.f.col
        c = self.f.ch
        if c == "{":
            return self._single(LCURLY, line, col)
        if c == "}":
            return self._single(RCURLY, line, col)
        if c == "[":
            return self._single(LBRACKET, line, col)
        if c == "]":
            return self._single(RBRACKET, line, col)
        if c == "/":
            p = self._peek()
            if _is_letter(p):
                self._read()
                return Token(BINDER, "/" + self._ident(), line, col)
            if p == "*":
                err = self._block_comment()
                if err:
                    return Token(ERROR, err, line, col)
                return self.next_token()
            return self._single(ILLEGAL, line, col)
        if c == '"':
            lit, err = self._string()
            return Token(ILLEGAL if err else STRING, lit, line, col)
        if c == "%":
            while self.f.ch not in ("\n", ""):
                self._read()
            return self.next_token()
        if c == "#":
            err = self._directive()
            if err:
                return Token(ERROR, err, line, col)
            return self.next_token()
        if c == "":
            return Token(EOF, "", line, col)
        if _is_letter(c):
            lit = self._ident()
            return Token(BOOLEAN if lit in ("true", "false") else IDENT, lit, line, col)
        if _is_digit(c) or c == "-":
            lit, typ = self._number()
            return Token(typ, lit, line, col)
        return self._single(ILLEGAL, line, col)

    def _block_comment(self):
        self._read()
        self._read()
        while True:
            if self.f.ch == "":
                return "unterminated block comment"
            if self.f.ch == "*" and self._peek() == "/":
                self._read()
                self._read()
                return None
            self._read()

    def _skip_inline_space(self):
        while self.f.ch in (" ", "\t"):
            self._read()

    def _directive(self):
        self._read()
        self._skip_inline_space()
        word = self._ident()
        if word == "include":
            self._skip_inline_space()
            if self.f.ch != '"':
                return "expected quoted filename after #include"
            name, err = self._string()
            if err:
                return "invalid #include filename: %s" % err
            return self._push_include(name)
        if word == "ifndef":
            self._skip_inline_space()
            name = self._ident()
            if not name:
                return "expected identifier after #ifndef"
            if name in self.defined:
                return self._skip_conditional()
            self.cond_depth += 1
            return None
        if word == "define":
            self._skip_inline_space()
            name = self._ident()
            if not name:
                return "expected identifier after #define"
            self.defined.add(name)
            return None
        if word == "endif":
            if self.cond_depth == 0:
                return "#endif without matching #ifndef"
            self.cond_depth -= 1
            return None
        return "unsupported preprocessor directive: #%s" % word

    def _push_include(self, name):
        d = os.path.dirname(self.f.file) if self.f.file else "."
        path = os.path.abspath(os.path.join(d, name))
        try:
            with open(path, "r") as fh:
                text = fh.read()
        except OSError as e:
            return "#include %s: %s" % (_go_quote(name), e.strerror or str(e))
        if path in self.active:
            return "#include %s: include cycle detected" % _go_quote(name)
        self.active.add(path)
        self.stack.append(self.f)
        self.f = _Frame(text, path)
        self._read()
        return None

    def _skip_conditional(self):
        depth = 1
        while depth > 0:
            if self.f.ch == "":
                return "unterminated #ifndef: missing #endif"
            if self.f.ch == "#":
                self._read()
                self._skip_inline_space()
                w = self._ident()
                if w == "ifndef":
                    depth += 1
                elif w == "endif":
                    depth -= 1
                continue
            self._read()
        return None

    def _ident(self):
        f = self.f
        out = []
        while _is_letter(self.f.ch) or _is_digit(self.f.ch) or self.f.ch in ("-", "_"):
            if self.f is not f:  # crossed an include boundary: stop like the Go slice would
                break
            out.append(self.f.ch)
            self._read()
        return "".join(out)

    def _number(self):
        out = []
        typ = INT
        if self.f.ch == "-":
            out.append("-")
            self._read()
        while _is_digit(self.f.ch):
            out.append(self.f.ch)
            self._read()
        if self.f.ch == ".":
            typ = FLOAT
            out.append(".")
            self._read()
            while _is_digit(self.f.ch):
                out.append(self.f.ch)
                self._read()
        if self.f.ch in ("e", "E"):
            typ = FLOAT
            out.append(self.f.ch)
            self._read()
            if self.f.ch in ("+", "-"):
                out.append(self.f.ch)
                self._read()
            while _is_digit(self.f.ch):
                out.append(self.f.ch)
                self._read()
        return "".join(out), typ

    def _string(self):
        out = []
        err = None
        self._read()
        while self.f.ch not in ('"', ""):
            if self.f.ch == "\\":
                self._read()
                c = self.f.ch
                if c == "n":
                    out.append("\n")
                elif c == "t":
                    out.append("\t")
                elif c == '"':
                    out.append('"')
                elif c == "\\":
                    out.append("\\")
                else:
                    err = "illegal escape sequence"
                    out.append("\\" + c)
            else:
                out.append(self.f.ch)
            self._read()
        if self.f.ch == '"':
            self._read()
        elif err is None:
            err = "unclosed string literal"
        return "".join(out), err


def _go_quote(s):
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'
