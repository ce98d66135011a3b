// psim_wire.cpp -- the wire format of a partisan peer connection (SURVEY.md
// 8(f) rank 4), so simulated nodes can exchange messages with real partisan
// nodes: every frame is {packet, 4} -- a 4-byte big-endian length
// (peer_service_client:214, the socket options of connect/2) -- around the
// encoding the connection's send path writes: handle_call({send_message, M})
// sends encode(M) (client:95, :130) = partisan_util:term_to_iolist/1
// (client:275-276, util:235-297) -- Erlang's external term format, version
// byte 131, with its own rules above the maps: atoms as SMALL_ATOM_EXT (115,
// a 1-byte length), tuples as SMALL_TUPLE_EXT, lists of bytes as STRING_EXT,
// other lists as LIST_EXT, and every other term -- the node_spec maps and
// everything inside them, integers -- through term_to_binary/1 (OTP 19-22:
// latin-1 atoms as ATOM_EXT, small maps with their keys in term order).  The
// receiver (server:172-182) takes any form; so does the decoder here.  (The
// client's hello, client:253-257, is default_encode = term_to_binary/1, and
// is not a record.)
//
// A message is the engine's 64-B record (psim_device.h Msg: dst, src,
// type | ttl << 8 | nex << 16, seq, a0, a1, a2, a3, ex[8]); the term is the
// one the reference's handler sends for it (hv = the HyParView manager,
// pt = partisan_plumtree_broadcast, xbot = the X-BOT manager):
//   JOIN               {join, Myself, Tag, Epoch}                          hv:506-510
//   FORWARD_JOIN       {forward_join, Peer, Tag, Epoch, TTL, Sender}       hv:743-748, :906-910
//   NEIGHBOR           {neighbor, Myself, Tag, DisconnectId, Peer}         hv:728-731
//   DISCONNECT         {disconnect, Myself, DisconnectId}                  hv:1493-1495
//   NEIGHBOR_REQUEST   {neighbor_request, Myself, high, Tag, Id, Exchange} hv:1700-1706
//   NEIGHBOR_ACCEPTED  {neighbor_accepted, Myself, Tag, Id, Exchange}      hv:1008-1012
//   NEIGHBOR_REJECTED  {neighbor_rejected, Myself, Exchange}               hv:1041-1043
//   SHUFFLE            {shuffle, Exchange, TTL, Sender}                    hv:594-597, :1110-1113
//   SHUFFLE_REPLY      {shuffle_reply, Exchange, Myself}                   hv:1127-1131
//   Plumtree           {forward_message, partisan_plumtree_broadcast, {'$gen_cast', Msg}}:
//                      send/3 (pt:633-638) calls cast_message/3, which wraps
//                      Msg as {'$gen_cast', Msg} (hv:147-154) for
//                      forward_message (hv:441-460); the receiver's
//                      process_forward sends it on as is (util:385-399)
//     BROADCAST        {broadcast, Id, Payload, Mod, Round, Root, From}    pt:398, :431
//     PRUNE            {prune, Root, From}                                 pt:372
//     IHAVE / IGNORED_IHAVE / GRAFT
//                      {i_have | ignored_i_have | graft, Id, Mod, Round, Root, From}  pt:381-385, :453
//     with the backend's heartbeat ids: Id = Payload = {RootName, Counter},
//     Mod = partisan_plumtree_backend (backend:81-83, :179-200)
//   X-BOT              {optimization | replace | switch, undefined, Old, I, C, D},
//                      {optimization_reply | replace_reply | switch_reply, Bool, Old, I, C, D}
//                                                                          xbot:1171-1314
// Tag is `undefined` (no tags configured); a DisconnectId {Epoch, Cnt} is
// the record's Epoch << 20 | Cnt; an Exchange is the list of ex[0 .. nex).
// Node id i is the node_spec #{name => '<prefix><i>@<host>', listen_addrs =>
// [#{ip => ip_base + i, port => port}], channels => [undefined],
// parallelism => 1} (partisan_peer_service_manager:myself/0 :71-76,
// partisan.hrl:14-19) -- a Plumtree identity without PSIM_MAP_BIT is the name
// atom alone.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/partisan_gpu_sim.h"

namespace {

enum : uint8_t {
    T_VERSION = 131, T_SMALL_INTEGER = 97, T_INTEGER = 98, T_ATOM = 100, T_SMALL_TUPLE = 104,
    T_LARGE_TUPLE = 105, T_NIL = 106, T_STRING = 107, T_LIST = 108, T_SMALL_BIG = 110,
    T_SMALL_ATOM = 115, T_MAP = 116, T_ATOM_UTF8 = 118, T_SMALL_ATOM_UTF8 = 119
};

constexpr uint32_t ID_EPOCH_SHIFT = 20;
constexpr uint32_t ID_CNT_MASK = (1u << ID_EPOCH_SHIFT) - 1;

const char* const kHvTags[] = {"join", "forward_join", "neighbor", "disconnect", "neighbor_request",
                               "neighbor_accepted", "neighbor_rejected", "shuffle", "shuffle_reply"};
const char* const kPtTags[] = {"broadcast", "prune", "i_have", "ignored_i_have", "graft"};
const char* const kXbTags[] = {"optimization", "optimization_reply", "replace", "replace_reply", "switch",
                               "switch_reply"};
const char* const kPlumtreeServer = "partisan_plumtree_broadcast";
const char* const kPlumtreeBackend = "partisan_plumtree_backend";

// ------------------------------------------------------------- encoder --
struct Enc {
    std::vector<uint8_t> b;
    // inside a term term_to_iolist/1 hands to term_to_binary/1 (a map)
    int in_map = 0;
    void u8(uint32_t v) { b.push_back((uint8_t)v); }
    void u16(uint32_t v) { u8(v >> 8); u8(v); }
    void u32(uint32_t v) { u16(v >> 16); u16(v); }
    // term_to_iolist_/1's atom clause (util:243-252): SMALL_ATOM_EXT up to
    // 255 characters; term_to_binary/1 inside a map: ATOM_EXT
    void atom(const std::string& s) {
        if (!in_map && s.size() <= 255) { u8(T_SMALL_ATOM); u8((uint32_t)s.size()); }
        else { u8(T_ATOM); u16((uint32_t)s.size()); }
        b.insert(b.end(), s.begin(), s.end());
    }
    void integer(int64_t v) {
        if (v >= 0 && v <= 255) { u8(T_SMALL_INTEGER); u8((uint32_t)v); return; }
        if (v >= INT32_MIN && v <= INT32_MAX) { u8(T_INTEGER); u32((uint32_t)(int32_t)v); return; }
        u8(T_SMALL_BIG);                                // (never needed by the records: ids are 32-bit)
        uint64_t m = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
        uint8_t d[8];
        uint32_t n = 0;
        while (m) { d[n++] = (uint8_t)m; m >>= 8; }
        u8(n); u8(v < 0 ? 1 : 0);
        for (uint32_t i = 0; i < n; i++) u8(d[i]);
    }
    void tuple(uint32_t n) { u8(T_SMALL_TUPLE); u8(n); }
    void list(uint32_t n) { u8(T_LIST); u32(n); }
    void nil() { u8(T_NIL); }
    void map(uint32_t n) { u8(T_MAP); u32(n); }
};

struct Names {
    std::string prefix, host;
    uint32_t ip_base, port;
    std::string name(uint32_t id) const { return prefix + std::to_string(id) + "@" + host; }
    // the id of a name atom, or PSIM_NONE
    uint32_t id_of(const std::string& s) const {
        if (s.size() <= prefix.size() + host.size() + 1 || s.compare(0, prefix.size(), prefix) != 0) return PSIM_NONE;
        const size_t at = s.size() - host.size() - 1;
        if (s[at] != '@' || s.compare(at + 1, std::string::npos, host) != 0) return PSIM_NONE;
        uint64_t v = 0;
        if (at == prefix.size()) return PSIM_NONE;
        for (size_t i = prefix.size(); i < at; i++) {
            if (s[i] < '0' || s[i] > '9') return PSIM_NONE;
            v = v * 10 + (uint32_t)(s[i] - '0');
            if (v >= PSIM_MAP_BIT) return PSIM_NONE;
        }
        if (at - prefix.size() > 1 && s[prefix.size()] == '0') return PSIM_NONE;   // (no leading zeros)
        return (uint32_t)v;
    }
};

// node_spec(): a map with its keys in term order (channels < listen_addrs <
// name < parallelism; ip < port)
void node_spec(Enc& e, const Names& nm, uint32_t id) {
    e.in_map++;                                       // (term_to_iolist_'s fallback clause, util:288-291)
    e.map(4);
    e.atom("channels"); e.list(1); e.atom("undefined"); e.nil();
    e.atom("listen_addrs"); e.list(1);
    e.map(2);
    const uint32_t ip = nm.ip_base + id;
    e.atom("ip"); e.tuple(4); e.integer(ip >> 24); e.integer((ip >> 16) & 255); e.integer((ip >> 8) & 255); e.integer(ip & 255);
    e.atom("port"); e.integer(nm.port);
    e.nil();
    e.atom("name"); e.atom(nm.name(id));
    e.atom("parallelism"); e.integer(1);
    e.in_map--;
}
// a Plumtree peer identity: a node_spec map (PSIM_MAP_BIT) or the name atom
void identity(Enc& e, const Names& nm, uint32_t ident) {
    if (ident & PSIM_MAP_BIT) node_spec(e, nm, ident & ~PSIM_MAP_BIT);
    else e.atom(nm.name(ident));
}
void disconnect_id(Enc& e, uint32_t id) {
    e.tuple(2); e.integer(id >> ID_EPOCH_SHIFT); e.integer(id & ID_CNT_MASK);
}
void exchange(Enc& e, const Names& nm, const uint32_t* ex, uint32_t nex) {
    if (nex) {
        e.list(nex);
        for (uint32_t i = 0; i < nex; i++) node_spec(e, nm, ex[i]);
    }
    e.nil();
}

// the term of a record; false for a record no handler sends
bool encode_term(Enc& e, const Names& nm, const uint32_t* r) {
    const uint32_t dst = r[0], src = r[1], type = r[2] & 0xFF, ttl = (r[2] >> 8) & 0xFF, nex = (r[2] >> 16) & 0xFF;
    const uint32_t a0 = r[4], a1 = r[5], a2 = r[6], a3 = r[7];
    const uint32_t* ex = r + 8;
    if (nex > PSIM_EXCHANGE_CAP) return false;
    switch (type) {
    case PSIM_MSG_JOIN:
        e.tuple(4); e.atom(kHvTags[type]); node_spec(e, nm, src); e.atom("undefined"); e.integer(a0);
        return true;
    case PSIM_MSG_FORWARD_JOIN:
        e.tuple(6); e.atom(kHvTags[type]); node_spec(e, nm, a0); e.atom("undefined"); e.integer(a1);
        e.integer(ttl); node_spec(e, nm, src);
        return true;
    case PSIM_MSG_NEIGHBOR:
        e.tuple(5); e.atom(kHvTags[type]); node_spec(e, nm, src); e.atom("undefined"); disconnect_id(e, a0);
        node_spec(e, nm, dst);
        return true;
    case PSIM_MSG_DISCONNECT:
        e.tuple(3); e.atom(kHvTags[type]); node_spec(e, nm, src); disconnect_id(e, a0);
        return true;
    case PSIM_MSG_NEIGHBOR_REQUEST:
        e.tuple(6); e.atom(kHvTags[type]); node_spec(e, nm, src); e.atom("high"); e.atom("undefined");
        disconnect_id(e, a0); exchange(e, nm, ex, nex);
        return true;
    case PSIM_MSG_NEIGHBOR_ACCEPTED:
        e.tuple(5); e.atom(kHvTags[type]); node_spec(e, nm, src); e.atom("undefined"); disconnect_id(e, a0);
        exchange(e, nm, ex, nex);
        return true;
    case PSIM_MSG_NEIGHBOR_REJECTED:
        e.tuple(3); e.atom(kHvTags[type]); node_spec(e, nm, src); exchange(e, nm, ex, nex);
        return true;
    case PSIM_MSG_SHUFFLE:
        e.tuple(4); e.atom(kHvTags[type]); exchange(e, nm, ex, nex); e.integer(ttl); node_spec(e, nm, src);
        return true;
    case PSIM_MSG_SHUFFLE_REPLY:
        e.tuple(3); e.atom(kHvTags[type]); exchange(e, nm, ex, nex); node_spec(e, nm, src);
        return true;
    case PSIM_MSG_PT_BROADCAST: case PSIM_MSG_PT_PRUNE: case PSIM_MSG_PT_IHAVE: case PSIM_MSG_PT_IGNORED_IHAVE:
    case PSIM_MSG_PT_GRAFT: {
        if (a2 == PSIM_NONE) return false;               // (an IHAVE of a retired id has no root)
        const std::string root_name = nm.name(a2 & ~PSIM_MAP_BIT);
        e.tuple(3); e.atom("forward_message"); e.atom(kPlumtreeServer);
        e.tuple(2); e.atom("$gen_cast");                 // cast_message/3 (hv:147-154)
        const auto id = [&] { e.tuple(2); e.atom(root_name); e.integer(a0); };
        if (type == PSIM_MSG_PT_PRUNE) {
            e.tuple(3); e.atom(kPtTags[1]); identity(e, nm, a2); node_spec(e, nm, src);
        } else if (type == PSIM_MSG_PT_BROADCAST) {
            e.tuple(7); e.atom(kPtTags[0]); id(); id(); e.atom(kPlumtreeBackend); e.integer(a1);
            identity(e, nm, a2); node_spec(e, nm, src);
        } else {
            e.tuple(6); e.atom(kPtTags[type - PSIM_MSG_PT_BROADCAST]); id(); e.atom(kPlumtreeBackend); e.integer(a1);
            identity(e, nm, a2); node_spec(e, nm, src);
        }
        return true;
    }
    case PSIM_MSG_XBOT_OPTIMIZATION: case PSIM_MSG_XBOT_OPTIMIZATION_REPLY: case PSIM_MSG_XBOT_REPLACE:
    case PSIM_MSG_XBOT_REPLACE_REPLY: case PSIM_MSG_XBOT_SWITCH: case PSIM_MSG_XBOT_SWITCH_REPLY: {
        const uint32_t k = type - PSIM_MSG_XBOT_OPTIMIZATION;
        const bool reply = (k & 1) != 0;
        e.tuple(6); e.atom(kXbTags[k]);
        if (reply) e.atom(ttl ? "true" : "false"); else e.atom("undefined");
        node_spec(e, nm, a0); node_spec(e, nm, a1); node_spec(e, nm, a2);
        if (a3 == PSIM_NONE) e.atom("undefined"); else node_spec(e, nm, a3);
        return true;
    }
    default:
        return false;
    }
}

// ------------------------------------------------------------- decoder --
struct Term {
    enum Kind { INT, ATOM, TUPLE, LIST, MAP } kind = INT;
    int64_t i = 0;
    std::string a;
    std::vector<Term> k;        // tuple / list elements; map: key, value, key, value, ...
};

struct Dec {
    const uint8_t* p;
    size_t n, at = 0;
    bool ok = true;
    uint32_t u8() { if (at + 1 > n) { ok = false; return 0; } return p[at++]; }
    uint32_t u16() { uint32_t h = u8(); return (h << 8) | u8(); }
    uint32_t u32() { uint32_t h = u16(); return (h << 16) | u16(); }
    bool term(Term& t, int depth) {
        if (depth > 16) return ok = false;
        const uint32_t tag = u8();
        if (!ok) return false;
        switch (tag) {
        case T_SMALL_INTEGER: t.kind = Term::INT; t.i = u8(); return ok;
        case T_INTEGER: t.kind = Term::INT; t.i = (int32_t)u32(); return ok;
        case T_SMALL_BIG: {
            const uint32_t d = u8(), sign = u8();
            if (d > 8) return ok = false;
            uint64_t v = 0;
            for (uint32_t j = 0; j < d; j++) v |= (uint64_t)u8() << (8 * j);
            if (v > (uint64_t)INT64_MAX) return ok = false;
            t.kind = Term::INT; t.i = sign ? -(int64_t)v : (int64_t)v;
            return ok;
        }
        case T_ATOM: case T_ATOM_UTF8: case T_SMALL_ATOM: case T_SMALL_ATOM_UTF8: {
            const uint32_t len = (tag == T_SMALL_ATOM || tag == T_SMALL_ATOM_UTF8) ? u8() : u16();
            if (!ok || at + len > n) return ok = false;
            t.kind = Term::ATOM; t.a.assign((const char*)p + at, len); at += len;
            return true;
        }
        case T_SMALL_TUPLE: case T_LARGE_TUPLE: {
            const uint32_t m = tag == T_SMALL_TUPLE ? u8() : u32();
            if (!ok || m > 64) return ok = false;
            t.kind = Term::TUPLE; t.k.resize(m);
            for (uint32_t j = 0; j < m; j++) if (!term(t.k[j], depth + 1)) return false;
            return true;
        }
        case T_NIL: t.kind = Term::LIST; return true;
        case T_STRING: {                                  // a list of small integers
            const uint32_t m = u16();
            if (!ok || at + m > n) return ok = false;
            t.kind = Term::LIST; t.k.resize(m);
            for (uint32_t j = 0; j < m; j++) { t.k[j].kind = Term::INT; t.k[j].i = p[at++]; }
            return true;
        }
        case T_LIST: {
            const uint32_t m = u32();
            if (!ok || m > 64) return ok = false;
            t.kind = Term::LIST; t.k.resize(m);
            for (uint32_t j = 0; j < m; j++) if (!term(t.k[j], depth + 1)) return false;
            Term tail;
            if (!term(tail, depth + 1) || tail.kind != Term::LIST || !tail.k.empty()) return ok = false;   // proper lists
            return true;
        }
        case T_MAP: {
            const uint32_t m = u32();
            if (!ok || m > 16) return ok = false;
            t.kind = Term::MAP; t.k.resize(2 * m);
            for (uint32_t j = 0; j < 2 * m; j++) if (!term(t.k[j], depth + 1)) return false;
            return true;
        }
        default:
            return ok = false;
        }
    }
};

bool is_atom(const Term& t, const char* s) { return t.kind == Term::ATOM && t.a == s; }
bool as_u32(const Term& t, uint32_t& v, uint32_t max = 0xFFFFFFFFu) {
    if (t.kind != Term::INT || t.i < 0 || (uint64_t)t.i > max) return false;
    v = (uint32_t)t.i;
    return true;
}
// a node_spec map (its name key) -> id
bool spec_id(const Term& t, const Names& nm, uint32_t& id) {
    if (t.kind != Term::MAP) return false;
    for (size_t j = 0; j + 1 < t.k.size(); j += 2)
        if (is_atom(t.k[j], "name") && t.k[j + 1].kind == Term::ATOM) {
            id = nm.id_of(t.k[j + 1].a);
            return id != PSIM_NONE;
        }
    return false;
}
// a Plumtree identity: map -> id | PSIM_MAP_BIT, name atom -> id
bool ident(const Term& t, const Names& nm, uint32_t& v) {
    if (t.kind == Term::ATOM) { v = nm.id_of(t.a); return v != PSIM_NONE; }
    if (!spec_id(t, nm, v)) return false;
    v |= PSIM_MAP_BIT;
    return true;
}
bool dis_id(const Term& t, uint32_t& v) {
    uint32_t e, c;
    if (t.kind != Term::TUPLE || t.k.size() != 2 || !as_u32(t.k[0], e, (1u << 12) - 1) ||
        !as_u32(t.k[1], c, ID_CNT_MASK))
        return false;
    v = (e << ID_EPOCH_SHIFT) | c;
    return true;
}
bool exch(const Term& t, const Names& nm, uint32_t* rec) {
    if (t.kind != Term::LIST || t.k.size() > PSIM_EXCHANGE_CAP) return false;
    for (size_t j = 0; j < t.k.size(); j++)
        if (!spec_id(t.k[j], nm, rec[8 + j])) return false;
    rec[2] |= (uint32_t)t.k.size() << 16;
    return true;
}
// {RootName, Counter} of a heartbeat id
bool msg_id(const Term& t, const Names& nm, uint32_t& root, uint32_t& ctr) {
    return t.kind == Term::TUPLE && t.k.size() == 2 && t.k[0].kind == Term::ATOM &&
           (root = nm.id_of(t.k[0].a)) != PSIM_NONE && as_u32(t.k[1], ctr);
}

bool decode_term(const Term& t, const Names& nm, uint32_t dst, uint32_t* r) {
    if (t.kind != Term::TUPLE || t.k.empty() || t.k[0].kind != Term::ATOM) return false;
    const std::string& tag = t.k[0].a;
    const size_t m = t.k.size();
    const auto& k = t.k;
    auto set_type = [&](uint32_t ty, uint32_t ttl) { r[2] = ty | (ttl << 8); };
    for (uint32_t ty = 0; ty <= PSIM_MSG_SHUFFLE_REPLY; ty++) {
        if (tag != kHvTags[ty]) continue;
        uint32_t ttl = 0;
        switch (ty) {
        case PSIM_MSG_JOIN:
            if (m != 4 || !spec_id(k[1], nm, r[1]) || !is_atom(k[2], "undefined") || !as_u32(k[3], r[4])) return false;
            set_type(ty, 0); return true;
        case PSIM_MSG_FORWARD_JOIN:
            if (m != 6 || !spec_id(k[1], nm, r[4]) || !is_atom(k[2], "undefined") || !as_u32(k[3], r[5]) ||
                !as_u32(k[4], ttl, 255) || !spec_id(k[5], nm, r[1]))
                return false;
            set_type(ty, ttl); return true;
        case PSIM_MSG_NEIGHBOR: {
            uint32_t to;
            if (m != 5 || !spec_id(k[1], nm, r[1]) || !is_atom(k[2], "undefined") || !dis_id(k[3], r[4]) ||
                !spec_id(k[4], nm, to) || to != dst)
                return false;
            set_type(ty, 0); return true;
        }
        case PSIM_MSG_DISCONNECT:
            if (m != 3 || !spec_id(k[1], nm, r[1]) || !dis_id(k[2], r[4])) return false;
            set_type(ty, 0); return true;
        case PSIM_MSG_NEIGHBOR_REQUEST:
            if (m != 6 || !spec_id(k[1], nm, r[1]) || !is_atom(k[2], "high") || !is_atom(k[3], "undefined") ||
                !dis_id(k[4], r[4]))
                return false;
            set_type(ty, 0); return exch(k[5], nm, r);
        case PSIM_MSG_NEIGHBOR_ACCEPTED:
            if (m != 5 || !spec_id(k[1], nm, r[1]) || !is_atom(k[2], "undefined") || !dis_id(k[3], r[4])) return false;
            set_type(ty, 0); return exch(k[4], nm, r);
        case PSIM_MSG_NEIGHBOR_REJECTED:
            if (m != 3 || !spec_id(k[1], nm, r[1])) return false;
            set_type(ty, 0); return exch(k[2], nm, r);
        case PSIM_MSG_SHUFFLE:
            if (m != 4 || !as_u32(k[2], ttl, 255) || !spec_id(k[3], nm, r[1])) return false;
            set_type(ty, ttl); return exch(k[1], nm, r);
        case PSIM_MSG_SHUFFLE_REPLY:
            if (m != 3 || !spec_id(k[2], nm, r[1])) return false;
            set_type(ty, 0); return exch(k[1], nm, r);
        }
    }
    if (tag == "forward_message") {
        // {forward_message, partisan_plumtree_broadcast, {'$gen_cast', Msg}}
        if (m != 3 || !is_atom(k[1], kPlumtreeServer) || k[2].kind != Term::TUPLE || k[2].k.size() != 2 ||
            !is_atom(k[2].k[0], "$gen_cast") || k[2].k[1].kind != Term::TUPLE || k[2].k[1].k.empty() ||
            k[2].k[1].k[0].kind != Term::ATOM)
            return false;
        const auto& q = k[2].k[1].k;
        const std::string& pt = q[0].a;
        uint32_t root = 0, ctr = 0;
        if (pt == kPtTags[1]) {
            if (q.size() != 3 || !ident(q[1], nm, r[6]) || !spec_id(q[2], nm, r[1])) return false;
            set_type(PSIM_MSG_PT_PRUNE, 0); return true;
        }
        if (pt == kPtTags[0]) {
            uint32_t r2 = 0, c2 = 0;
            if (q.size() != 7 || !msg_id(q[1], nm, root, ctr) || !msg_id(q[2], nm, r2, c2) || r2 != root || c2 != ctr ||
                !is_atom(q[3], kPlumtreeBackend) || !as_u32(q[4], r[5]) || !ident(q[5], nm, r[6]) ||
                (r[6] & ~PSIM_MAP_BIT) != root || !spec_id(q[6], nm, r[1]) || ctr > 0xFFFFu)
                return false;
            r[4] = ctr;
            set_type(PSIM_MSG_PT_BROADCAST, 0); return true;
        }
        for (uint32_t j = 2; j < 5; j++) {
            if (pt != kPtTags[j]) continue;
            if (q.size() != 6 || !msg_id(q[1], nm, root, ctr) || !is_atom(q[2], kPlumtreeBackend) ||
                !as_u32(q[3], r[5]) || !ident(q[4], nm, r[6]) || (r[6] & ~PSIM_MAP_BIT) != root ||
                !spec_id(q[5], nm, r[1]) || ctr > 0xFFFFu)
                return false;
            r[4] = ctr;
            set_type(PSIM_MSG_PT_BROADCAST + j, 0); return true;
        }
        return false;
    }
    for (uint32_t j = 0; j < 6; j++) {
        if (tag != kXbTags[j]) continue;
        const bool reply = (j & 1) != 0;
        uint32_t ans = 0;
        if (m != 6) return false;
        if (reply) {
            if (is_atom(k[1], "true")) ans = 1;
            else if (!is_atom(k[1], "false")) return false;
        } else if (!is_atom(k[1], "undefined")) {
            return false;
        }
        if (!spec_id(k[2], nm, r[4]) || !spec_id(k[3], nm, r[5]) || !spec_id(k[4], nm, r[6])) return false;
        if (is_atom(k[5], "undefined")) r[7] = PSIM_NONE;
        else if (!spec_id(k[5], nm, r[7])) return false;
        // (the sender is not in the term: the connection's peer, the caller's
        // to fill; here the node the protocol step comes from)
        const uint32_t from[6] = {r[5], r[6], r[6], r[7], r[7], r[4]};
        r[1] = from[j];
        set_type(PSIM_MSG_XBOT_OPTIMIZATION + j, ans);
        return true;
    }
    return false;
}

bool names_of(const psim_wire_names* w, Names& nm) {
    if (!w || !w->prefix || !w->host || !w->host[0]) return false;
    nm.prefix = w->prefix; nm.host = w->host; nm.ip_base = w->ip_base; nm.port = w->port;
    return true;
}

}  // namespace

extern "C" {

int psim_wire_encode(const uint32_t rec[16], const psim_wire_names* names, uint8_t* buf, size_t cap, size_t* len) {
    Names nm;
    if (!rec || !len || !names_of(names, nm)) return PSIM_EINVAL;
    Enc e;
    e.b.reserve(1024);
    e.u32(0);                                         // the {packet, 4} length, filled below
    e.u8(T_VERSION);
    if (!encode_term(e, nm, rec)) return PSIM_EINVAL;
    const size_t body = e.b.size() - 4;
    e.b[0] = (uint8_t)(body >> 24); e.b[1] = (uint8_t)(body >> 16); e.b[2] = (uint8_t)(body >> 8); e.b[3] = (uint8_t)body;
    *len = e.b.size();
    if (buf && cap >= e.b.size()) memcpy(buf, e.b.data(), e.b.size());
    return PSIM_OK;
}

int psim_wire_decode(const uint8_t* buf, size_t len, const psim_wire_names* names, uint32_t dst, uint32_t rec[16],
                     size_t* used) {
    Names nm;
    if (!buf || !rec || !used || !names_of(names, nm)) return PSIM_EINVAL;
    *used = 0;
    if (len < 4) return PSIM_ERANGE;                  // an incomplete frame: read more
    const size_t body = ((size_t)buf[0] << 24) | ((size_t)buf[1] << 16) | ((size_t)buf[2] << 8) | buf[3];
    if (len < 4 + body) return PSIM_ERANGE;
    Dec d{buf + 4, body};
    if (d.u8() != T_VERSION) return PSIM_EINVAL;
    Term t;
    if (!d.term(t, 0) || d.at != body) return PSIM_EINVAL;
    uint32_t r[16] = {};
    r[0] = dst;
    if (!decode_term(t, nm, dst, r)) return PSIM_EINVAL;
    memcpy(rec, r, sizeof r);
    *used = 4 + body;
    return PSIM_OK;
}

}  // extern "C"
