"""A small, independent encoder of Erlang's external term format (version
131), written from the published format description (erts "External Term
Format") for the tests of the wire codec: term_to_binary/1 as OTP 19-22
writes it -- latin-1 atoms as ATOM_EXT, integers as SMALL_INTEGER_EXT /
INTEGER_EXT, lists of small integers as STRING_EXT, small maps with their
keys in term order.  Test infrastructure only."""
import struct


class Atom(str):
    pass


def _key(t):
    # Erlang term order between the kinds used here: number < atom < tuple < map < list
    if isinstance(t, int):
        return (0, t)
    if isinstance(t, Atom):
        return (1, str(t))
    raise TypeError(t)


def _enc(t, out):
    if isinstance(t, Atom):
        b = str(t).encode("latin-1")
        out += bytes([100]) + struct.pack(">H", len(b)) + b
    elif isinstance(t, bool):
        raise TypeError("use Atom('true') / Atom('false')")
    elif isinstance(t, int):
        if 0 <= t <= 255:
            out += bytes([97, t])
        else:
            out += bytes([98]) + struct.pack(">i", t)
    elif isinstance(t, tuple):
        out += bytes([104, len(t)])
        for x in t:
            _enc(x, out)
    elif isinstance(t, list):
        if not t:
            out += bytes([106])
        elif all(isinstance(x, int) and not isinstance(x, bool) and 0 <= x <= 255 for x in t):
            out += bytes([107]) + struct.pack(">H", len(t)) + bytes(t)
        else:
            out += bytes([108]) + struct.pack(">I", len(t))
            for x in t:
                _enc(x, out)
            out += bytes([106])
    elif isinstance(t, dict):
        out += bytes([116]) + struct.pack(">I", len(t))
        for k in sorted(t, key=_key):
            _enc(k, out)
            _enc(t[k], out)
    else:
        raise TypeError(t)


def _iolist(t, out):
    """partisan_util:term_to_iolist_/1 (util:238-291), restated: atoms as
    SMALL_ATOM_EXT, tuples as SMALL_TUPLE_EXT, lists of bytes as STRING_EXT,
    other lists as LIST_EXT, anything else (maps, integers) via
    term_to_binary/1."""
    if isinstance(t, Atom) and len(str(t)) <= 255:
        b = str(t).encode("latin-1")
        out += bytes([115, len(b)]) + b
    elif isinstance(t, tuple):
        out += bytes([104, len(t)])
        for x in t:
            _iolist(x, out)
    elif isinstance(t, list):
        if not t:
            out += bytes([106])
        elif all(isinstance(x, int) and not isinstance(x, bool) and 0 <= x <= 255 for x in t):
            out += bytes([107]) + struct.pack(">H", len(t)) + bytes(t)
        else:
            out += bytes([108]) + struct.pack(">I", len(t))
            for x in t:
                _iolist(x, out)
            out += bytes([106])
    else:
        _enc(t, out)


def term_to_iolist(t):
    """The bytes of partisan_util:term_to_iolist/1: what a partisan
    connection writes for a message (peer_service_client:95, :130, :275)."""
    out = bytearray([131])
    _iolist(t, out)
    return bytes(out)


def term_to_binary(t):
    out = bytearray([131])
    _enc(t, out)
    return bytes(out)


def packet4(b):
    return struct.pack(">I", len(b)) + b
