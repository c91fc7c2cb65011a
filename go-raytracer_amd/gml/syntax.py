"""GML token groups and parser (internal/gml/expr.go, parser.go)."""
from . import lexer as L
from .gofmt import format_float


class IDMapping:
    """environment.go:90-112: ids are assigned 1, 2, ... in first-seen order."""

    def __init__(self):
        self.name_id = {}
        self.id_name = {}
        self.max_id = 0

    def get_or_create(self, name):
        i = self.name_id.get(name)
        if i is None:
            self.max_id += 1
            i = self.max_id
            self.name_id[name] = i
            self.id_name[i] = name
        return i

    def clone(self):
        m = IDMapping()
        m.name_id = dict(self.name_id)
        m.id_name = dict(self.id_name)
        m.max_id = self.max_id
        return m


class Tok:
    __slots__ = ("pos",)


class Identifier(Tok):
    __slots__ = ("name", "id")

    def __init__(self, name, id_, pos):
        self.name, self.id, self.pos = name, id_, pos


class Binder(Tok):
    __slots__ = ("name", "id")

    def __init__(self, name, id_, pos):
        self.name, self.id, self.pos = name, id_, pos


class IntLit(Tok):
    __slots__ = ("value",)

    def __init__(self, v, pos):
        self.value, self.pos = v, pos


class FloatLit(Tok):
    __slots__ = ("value",)

    def __init__(self, v, pos):
        self.value, self.pos = v, pos


class BoolLit(Tok):
    __slots__ = ("value",)

    def __init__(self, v, pos):
        self.value, self.pos = v, pos


class StringLit(Tok):
    __slots__ = ("value",)

    def __init__(self, v, pos):
        self.value, self.pos = v, pos


class Function(Tok):
    __slots__ = ("body",)

    def __init__(self, body, pos):
        self.body, self.pos = body, pos


class Array(Tok):
    __slots__ = ("elements",)

    def __init__(self, elements, pos):
        self.elements, self.pos = elements, pos


def _go_quote(s):
    out = ['"']
    for ch in s:
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\t":
            out.append("\\t")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def token_debug_string(g):
    """TokenGroupDebugString (expr.go:130-152)."""
    if isinstance(g, IntLit):
        return str(g.value)
    if isinstance(g, FloatLit):
        return format_float(g.value)
    if isinstance(g, BoolLit):
        return "true" if g.value else "false"
    if isinstance(g, StringLit):
        return _go_quote(g.value)
    if isinstance(g, Identifier):
        return g.name
    if isinstance(g, Binder):
        return "/" + g.name
    if isinstance(g, Function):
        return "{ " + token_list_string(g.body) + " }"
    if isinstance(g, Array):
        return "[ " + token_list_string(g.elements) + " ]"
    raise TypeError(g)


def token_list_string(tl):
    return " ".join(token_debug_string(t) for t in tl)


class ParseError(Exception):
    pass


_STARTS = (L.LBRACKET, L.LCURLY, L.IDENT, L.INT, L.FLOAT, L.STRING, L.BINDER, L.BOOLEAN)


class Parser:
    """Recursive descent over token groups (parser.go:43-226)."""

    def __init__(self, lexer, idmap):
        self.lx = lexer
        self.ids = idmap
        self.cur = None

    def _adv(self):
        t = self.cur
        self.cur = self.lx.next_token()
        return t

    def parse(self):
        self._adv()
        lst = self._list()
        if self.cur.type == L.ERROR:
            raise ParseError("%d:%d: %s" % (self.cur.line, self.cur.col, self.cur.literal))
        if self.cur.type != L.EOF:
            raise ParseError("%d:%d: unexpected token: %s, expected end of input"
                             % (self.cur.line, self.cur.col, L.NAMES[self.cur.type]))
        return lst

    def _consume(self, typ):
        if self.cur.type == L.ERROR:
            raise ParseError("%d:%d: %s" % (self.cur.line, self.cur.col, self.cur.literal))
        if self.cur.type != typ:
            raise ParseError("%d:%d: expected %s, got %s" % (self.cur.line, self.cur.col, L.NAMES[typ],
                                                             L.NAMES[self.cur.type]))
        self._adv()

    def _list(self):
        out = []
        while self.cur.type in _STARTS:
            out.append(self._group())
        return out

    def _group(self):
        t = self.cur
        pos = (t.line, t.col)
        if t.type == L.LBRACKET:
            self._consume(L.LBRACKET)
            els = self._list()
            self._consume(L.RBRACKET)
            return Array(els, pos)
        if t.type == L.LCURLY:
            self._consume(L.LCURLY)
            body = self._list()
            self._consume(L.RCURLY)
            return Function(body, pos)
        self._adv()
        if t.type == L.IDENT:
            return Identifier(t.literal, self.ids.get_or_create(t.literal), pos)
        if t.type == L.INT:
            try:
                v = int(t.literal, 10)
            except ValueError:
                raise ParseError("%d:%d: could not parse number: %s" % (t.line, t.col, t.literal))
            if not (-(1 << 63) <= v < (1 << 63)):
                raise ParseError("%d:%d: could not parse number: %s" % (t.line, t.col, t.literal))
            return IntLit(v, pos)
        if t.type == L.FLOAT:
            try:
                v = float(t.literal)
            except ValueError:
                raise ParseError("%d:%d: could not parse number: %s" % (t.line, t.col, t.literal))
            return FloatLit(v, pos)
        if t.type == L.STRING:
            return StringLit(t.literal, pos)
        if t.type == L.BINDER:
            name = t.literal[1:]
            return Binder(name, self.ids.get_or_create(name), pos)
        if t.type == L.BOOLEAN:
            return BoolLit(t.literal == "true", pos)
        raise ParseError("%d:%d: unexpected token: %s" % (t.line, t.col, L.NAMES[t.type]))


def parse_text(text, idmap, file=""):
    return Parser(L.Lexer(text, file), idmap).parse()


def parse_file(path, idmap):
    return Parser(L.Lexer.from_file(path), idmap).parse()
