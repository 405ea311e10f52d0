// trace.cpp — zlib + a minimal JSON reader for the fixed josephg trace schema.
#include "trace.hpp"

#include <zlib.h>

#include <cstdio>
#include <cstring>

#include "store.hpp"
#include "util.hpp"

namespace crdt {

namespace {

std::string gunzip_file(const std::string& path, std::string& out) {
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) return "cannot open " + path;
    gzbuffer(f, 1 << 20);
    char buf[1 << 16];
    for (;;) {
        int k = gzread(f, buf, sizeof buf);
        if (k < 0) {
            int e;
            std::string m = gzerror(f, &e);
            gzclose(f);
            return "gzip error in " + path + ": " + m;
        }
        if (k == 0) break;
        out.append(buf, (size_t)k);
    }
    gzclose(f);
    return "";
}

struct Reader {
    const char* p;
    const char* e;
    std::string err;

    void ws() {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool eat(char c) {
        ws();
        if (p < e && *p == c) { ++p; return true; }
        return false;
    }
    bool expect(char c) {
        if (eat(c)) return true;
        if (err.empty()) err = std::string("expected '") + c + "'";
        return false;
    }
    static int hexv(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    bool hex4(uint32_t& v) {
        if (e - p < 4) return false;
        v = 0;
        for (int i = 0; i < 4; ++i) {
            int h = hexv(p[i]);
            if (h < 0) return false;
            v = (v << 4) | (uint32_t)h;
        }
        p += 4;
        return true;
    }
    // JSON string -> UTF-8 appended to out.
    bool str(std::string& out) {
        if (!expect('"')) return false;
        while (p < e) {
            const char* run = p;
            while (p < e && *p != '"' && *p != '\\') ++p;
            out.append(run, (size_t)(p - run));
            if (p >= e) break;
            if (*p == '"') { ++p; return true; }
            ++p;  // backslash
            if (p >= e) break;
            char c = *p++;
            switch (c) {
                case '"': out.push_back('"'); break;
                case '\\': out.push_back('\\'); break;
                case '/': out.push_back('/'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    uint32_t u;
                    if (!hex4(u)) { err = "bad \\u escape"; return false; }
                    if (u >= 0xD800 && u < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        const char* save = p;
                        p += 2;
                        uint32_t lo;
                        if (hex4(lo) && lo >= 0xDC00 && lo < 0xE000) {
                            u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
                        } else {
                            p = save;
                        }
                    }
                    char b[4];
                    out.append(b, utf8_put(u, b));
                    break;
                }
                default: err = "bad escape"; return false;
            }
        }
        err = "unterminated string";
        return false;
    }
    bool uint(uint64_t& v) {
        ws();
        if (p >= e || *p < '0' || *p > '9') { err = "expected unsigned integer"; return false; }
        v = 0;
        while (p < e && *p >= '0' && *p <= '9') v = v * 10 + (uint64_t)(*p++ - '0');
        if (p < e && (*p == '.' || *p == 'e' || *p == 'E')) { err = "non-integer position"; return false; }
        return true;
    }
    bool skip_value() {
        ws();
        if (p >= e) { err = "eof"; return false; }
        char c = *p;
        if (c == '"') { std::string tmp; return str(tmp); }
        if (c == '{' || c == '[') {
            char close = c == '{' ? '}' : ']';
            ++p;
            if (eat(close)) return true;
            for (;;) {
                if (c == '{') {
                    std::string k;
                    if (!str(k) || !expect(':')) return false;
                }
                if (!skip_value()) return false;
                if (eat(',')) continue;
                return expect(close);
            }
        }
        while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n') ++p;
        return true;
    }
};

}  // namespace

std::string parse_trace_json(const char* data, size_t n, Trace& t) {
    Reader r{data, data + n, ""};
    t = Trace{};
    bool have_txns = false;
    if (!r.expect('{')) return r.err;
    if (!r.eat('}')) {
        for (;;) {
            std::string key;
            if (!r.str(key) || !r.expect(':')) return r.err;
            if (key == "startContent") {
                if (!r.str(t.start_content)) return r.err;
            } else if (key == "endContent") {
                if (!r.str(t.end_content)) return r.err;
            } else if (key == "txns") {
                have_txns = true;
                if (!r.expect('[')) return r.err;
                if (!r.eat(']')) {
                    for (;;) {  // txn object
                        if (!r.expect('{')) return r.err;
                        if (!r.eat('}')) {
                            for (;;) {
                                std::string tk;
                                if (!r.str(tk) || !r.expect(':')) return r.err;
                                if (tk == "patches") {
                                    if (!r.expect('[')) return r.err;
                                    if (!r.eat(']')) {
                                        for (;;) {
                                            Patch pt{};
                                            if (!r.expect('[') || !r.uint(pt.pos) ||
                                                !r.expect(',') || !r.uint(pt.del) ||
                                                !r.expect(','))
                                                return r.err;
                                            pt.ins_off = t.ins.size();
                                            if (!r.str(t.ins)) return r.err;
                                            pt.ins_len = t.ins.size() - pt.ins_off;
                                            if (!r.expect(']')) return r.err;
                                            t.patches.push_back(pt);
                                            if (r.eat(',')) continue;
                                            if (!r.expect(']')) return r.err;
                                            break;
                                        }
                                    }
                                } else if (!r.skip_value()) {
                                    return r.err;
                                }
                                if (r.eat(',')) continue;
                                if (!r.expect('}')) return r.err;
                                break;
                            }
                        }
                        t.txn_end.push_back((uint32_t)t.patches.size());
                        if (r.eat(',')) continue;
                        if (!r.expect(']')) return r.err;
                        break;
                    }
                }
            } else if (!r.skip_value()) {
                return r.err;
            }
            if (r.eat(',')) continue;
            if (!r.expect('}')) return r.err;
            break;
        }
    }
    if (!have_txns) return "trace has no txns";
    return "";
}

std::string load_trace(const std::string& path, Trace& out) {
    if (is_trace_bin(path)) return load_trace_bin(path, out);  // trace cache (store.hpp)
    std::string raw;
    std::string e = gunzip_file(path, raw);
    if (!e.empty()) return e;
    e = parse_trace_json(raw.data(), raw.size(), out);
    if (!e.empty()) return path + ": " + e;
    return "";
}

// chars_to_bytes: replay the patches over a gap buffer holding each codepoint's extra UTF-8
// bytes (len - 1); the byte offset of codepoint position p is p + (extra bytes before p), and
// the gap is always moved to p, so that sum is maintained incrementally.
std::string chars_to_bytes(Trace& t) {
    if (t.byte_offsets) return "";
    std::vector<uint8_t> buf;  // extra bytes per codepoint; gap = [gs, ge)
    size_t gs = 0, ge = 0;
    uint64_t extra_before = 0;
    auto len = [&] { return buf.size() - (ge - gs); };
    auto reserve = [&](size_t need) {
        if (ge - gs >= need) return;
        size_t ncap = (len() + need) * 2 + 64;
        std::vector<uint8_t> nb(ncap);
        size_t tail = buf.size() - ge;
        if (gs) std::memcpy(nb.data(), buf.data(), gs);  // (buf may still be empty: no null src)
        if (tail) std::memcpy(nb.data() + ncap - tail, buf.data() + ge, tail);
        buf.swap(nb);
        ge = ncap - tail;
    };
    auto move_to = [&](size_t pos) {
        while (gs > pos) { --gs; --ge; buf[ge] = buf[gs]; extra_before -= buf[ge]; }
        while (gs < pos) { buf[gs] = buf[ge]; extra_before += buf[gs]; ++gs; ++ge; }
    };
    auto insert_text = [&](const char* s, size_t n) {
        size_t cps = utf8_count(s, n);
        reserve(cps);
        const unsigned char* q = (const unsigned char*)s;
        for (size_t i = 0; i < n; ++i) {
            if ((q[i] & 0xC0) != 0x80) { buf[gs++] = 0; extra_before += 0; }
            else { buf[gs - 1]++; extra_before++; }
        }
    };
    insert_text(t.start_content.data(), t.start_content.size());
    move_to(0);
    for (Patch& p : t.patches) {
        if (p.pos > len() || p.del > len() - p.pos) return "patch out of range";
        move_to(p.pos);
        uint64_t bpos = p.pos + extra_before;
        uint64_t dextra = 0;
        for (uint64_t k = 0; k < p.del; ++k) dextra += buf[ge + k];
        ge += p.del;
        uint64_t bdel = p.del + dextra;
        insert_text(t.ins.data() + p.ins_off, p.ins_len);
        p.pos = bpos;
        p.del = bdel;
    }
    t.byte_offsets = true;
    return "";
}

}  // namespace crdt
