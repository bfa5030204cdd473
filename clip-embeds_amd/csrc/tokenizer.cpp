// CLIP byte-level BPE tokenizer on the host (C++17), behind the C ABI in include/clipembed.h.
//
// Restates open_clip's SimpleTokenizer (open_clip/src/open_clip/tokenizer.py:133-265):
//   * bytes_to_unicode (tokenizer.py:31-51): the 188 printable Latin-1 bytes map to themselves,
//     the other 68 to U+0100.. in byte order;
//   * vocabulary (tokenizer.py:144-156): 256 byte symbols, the same with "</w>", one entry per
//     merge (lines 1 .. 48894 of the merges file), then <start_of_text>, <end_of_text>, extras;
//   * pre-tokenizer (tokenizer.py:159-163): specials | 's 't 're 've 'm 'll 'd | [\p{L}]+ | [\p{N}] |
//     [^\s\p{L}\p{N}]+ , IGNORECASE, ordered alternation, whitespace skipped; Unicode classes from
//     unicode_tables.h (generated from the `regex` module the reference uses);
//   * bpe (tokenizer.py:172-211): last symbol carries "</w>", repeatedly merge every
//     non-overlapping occurrence (left to right) of the lowest-ranked adjacent pair;
//   * __call__ (tokenizer.py:226-265): [SOT] + ids + [EOT], truncate to context_length with the
//     last id forced to EOT, zero padding.
// Text cleaning (ftfy / html.unescape / whitespace / lower, tokenizer.py:66-90) stays in the
// Python host layer (clipembed/tokenizer.py), which hands this code the cleaned UTF-8 text.
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "unicode_tables.h"

namespace {

bool in_ranges(const CpRange* r, int n, uint32_t cp) {
    int lo = 0, hi = n - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (cp < r[mid].lo) hi = mid - 1;
        else if (cp > r[mid].hi) lo = mid + 1;
        else return true;
    }
    return false;
}
bool is_letter(uint32_t cp) { return cp < 128 ? ((cp | 32) - 'a' < 26u) : in_ranges(kLetter, kLetter_n, cp); }
bool is_number(uint32_t cp) { return cp < 128 ? (cp - '0' < 10u) : in_ranges(kNumber, kNumber_n, cp); }
bool is_space(uint32_t cp) { return in_ranges(kSpace, kSpace_n, cp); }

void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) {
        s += (char)cp;
    } else if (cp < 0x800) {
        s += (char)(0xC0 | (cp >> 6));
        s += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
        s += (char)(0xE0 | (cp >> 12));
        s += (char)(0x80 | ((cp >> 6) & 0x3F));
        s += (char)(0x80 | (cp & 0x3F));
    } else {
        s += (char)(0xF0 | (cp >> 18));
        s += (char)(0x80 | ((cp >> 12) & 0x3F));
        s += (char)(0x80 | ((cp >> 6) & 0x3F));
        s += (char)(0x80 | (cp & 0x3F));
    }
}

// Decode one code point of valid UTF-8 at s[i]; returns its byte length (the Python host layer
// only passes str-encoded text, so the input is always valid).
int next_cp(const std::string& s, size_t i, uint32_t& cp) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) { cp = c; return 1; }
    if ((c >> 5) == 6 && i + 1 < s.size()) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); return 2; }
    if ((c >> 4) == 14 && i + 2 < s.size()) {
        cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
        return 3;
    }
    if ((c >> 3) == 30 && i + 3 < s.size()) {
        cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
        return 4;
    }
    cp = 0xFFFD;
    return 1;
}

uint32_t ascii_lower(uint32_t cp) { return (cp >= 'A' && cp <= 'Z') ? cp + 32 : cp; }

}  // namespace

struct ce_tokenizer {
    std::string byte_sym[256];                       // bytes_to_unicode, as UTF-8
    std::unordered_map<uint32_t, int> sym_byte;      // inverse (code point -> byte)
    std::unordered_map<std::string, int32_t> encoder;
    std::vector<std::string> decoder;
    std::unordered_map<std::string, int> ranks;      // "a b" -> merge rank
    std::vector<std::string> specials;               // matched first by the pre-tokenizer
    std::unordered_map<std::string, std::vector<int32_t>> cache;
    std::mutex mu;                                   // guards cache (calls may come from threads)
    int32_t sot = 0, eot = 0;

    // --- pre-tokenizer: byte ranges of the pattern's matches, in order ---
    // Alternation order as in tokenizer.py:160-163; under IGNORECASE the contraction letters match
    // either case (and 's' also U+017F, LATIN SMALL LETTER LONG S, which case-folds to 's').
    size_t match_at(const std::string& t, size_t i) const {
        for (const std::string& sp : specials) {
            if (t.size() - i < sp.size()) continue;
            bool ok = true;   // specials are ASCII: ASCII case-insensitive compare
            for (size_t k = 0; k < sp.size() && ok; ++k)
                ok = ascii_lower((unsigned char)t[i + k]) == ascii_lower((unsigned char)sp[k]);
            if (ok) return sp.size();
        }
        uint32_t cp;
        const int n0 = next_cp(t, i, cp);
        if (cp == '\'') {
            static const char* contr[] = {"s", "t", "re", "ve", "m", "ll", "d"};
            for (const char* c : contr) {
                size_t j = i + 1;
                bool ok = true;
                for (const char* q = c; *q && ok; ++q) {
                    if (j >= t.size()) { ok = false; break; }
                    uint32_t x;
                    const int n = next_cp(t, j, x);
                    ok = ascii_lower(x) == (uint32_t)*q || (*q == 's' && x == 0x17F);
                    j += n;
                }
                if (ok) return j - i;
            }
        }
        if (is_letter(cp)) {
            size_t j = i + n0;
            while (j < t.size()) {
                uint32_t x;
                const int n = next_cp(t, j, x);
                if (!is_letter(x)) break;
                j += n;
            }
            return j - i;
        }
        if (is_number(cp)) return n0;
        if (!is_space(cp)) {
            size_t j = i + n0;
            while (j < t.size()) {
                uint32_t x;
                const int n = next_cp(t, j, x);
                if (is_space(x) || is_letter(x) || is_number(x)) break;
                j += n;
            }
            return j - i;
        }
        return 0;
    }

    // --- BPE of one pre-token (tokenizer.py:172-211) ---
    void bpe(const std::string& piece, std::vector<int32_t>& out) {
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = cache.find(piece);
            if (it != cache.end()) {
                out.insert(out.end(), it->second.begin(), it->second.end());
                return;
            }
        }
        std::vector<int32_t> ids;
        auto sp = encoder.find(piece);
        bool is_special = false;
        for (const std::string& s : specials) is_special |= s == piece;
        if (is_special && sp != encoder.end()) {
            ids.push_back(sp->second);       // cache seeded with the specials (tokenizer.py:158)
        } else {
            std::vector<std::string> word;
            for (unsigned char b : piece) word.push_back(byte_sym[b]);
            word.back() += "</w>";
            std::string key;
            while (word.size() > 1) {
                int best = -1;
                size_t bi = 0;
                for (size_t k = 0; k + 1 < word.size(); ++k) {
                    key.assign(word[k]).append(" ").append(word[k + 1]);
                    auto r = ranks.find(key);
                    if (r != ranks.end() && (best < 0 || r->second < best)) {
                        best = r->second;
                        bi = k;
                    }
                }
                if (best < 0) break;
                const std::string first = word[bi], second = word[bi + 1];
                std::vector<std::string> nw;
                nw.reserve(word.size());
                for (size_t k = 0; k < word.size();) {
                    if (k + 1 < word.size() && word[k] == first && word[k + 1] == second) {
                        nw.push_back(first + second);
                        k += 2;
                    } else {
                        nw.push_back(word[k]);
                        k += 1;
                    }
                }
                word.swap(nw);
            }
            for (const std::string& w : word) {
                auto e = encoder.find(w);
                ids.push_back(e == encoder.end() ? 0 : e->second);
            }
        }
        out.insert(out.end(), ids.begin(), ids.end());
        std::lock_guard<std::mutex> g(mu);
        cache.emplace(piece, std::move(ids));
    }

    void encode(const std::string& text, std::vector<int32_t>& out) {
        size_t i = 0;
        while (i < text.size()) {
            const size_t n = match_at(text, i);
            if (n == 0) {
                uint32_t cp;
                i += next_cp(text, i, cp);    // whitespace: not part of any match
                continue;
            }
            bpe(text.substr(i, n), out);
            i += n;
        }
    }
};

namespace {

thread_local std::string g_tok_err;
int tok_fail(const char* msg) {
    g_tok_err = msg;
    return 1;
}

}  // namespace

extern "C" {

const char* ce_tokenizer_last_error() { return g_tok_err.c_str(); }

int ce_tokenizer_create(const char* merges, size_t len, const char* const* extra_special, int n_extra,
                        ce_tokenizer** out) {
    if (!merges || !out) return tok_fail("ce_tokenizer_create: null argument");
    auto* t = new ce_tokenizer();
    // bytes_to_unicode (tokenizer.py:42-51)
    std::vector<int> bs, cs;
    for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
    for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
    for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
    cs = bs;
    int n = 0;
    for (int b = 0; b < 256; ++b) {
        bool have = false;
        for (int x : bs) have |= x == b;
        if (!have) {
            bs.push_back(b);
            cs.push_back(256 + n++);
        }
    }
    for (size_t k = 0; k < bs.size(); ++k) {
        put_utf8(t->byte_sym[bs[k]], (uint32_t)cs[k]);
        t->sym_byte[(uint32_t)cs[k]] = bs[k];
    }
    // vocabulary in the reference's order: byte symbols in bytes_to_unicode().values() order
    // (= the bs order above), then the same with </w>, then merges, then specials
    std::vector<std::string> vocab;
    for (size_t k = 0; k < bs.size(); ++k) vocab.push_back(t->byte_sym[bs[k]]);
    for (size_t k = 0; k < bs.size(); ++k) vocab.push_back(t->byte_sym[bs[k]] + "</w>");
    // merges = lines[1 : 49152 - 256 - 2 + 1]
    std::vector<std::string> lines;
    {
        size_t s = 0;
        const std::string all(merges, len);
        while (s <= all.size()) {
            size_t e = all.find('\n', s);
            if (e == std::string::npos) e = all.size();
            lines.push_back(all.substr(s, e - s));
            s = e + 1;
        }
    }
    const size_t last = std::min<size_t>(lines.size(), 49152 - 256 - 2 + 1);
    int rank = 0;
    for (size_t k = 1; k < last; ++k) {
        const std::string& l = lines[k];
        const size_t sp = l.find(' ');
        if (sp == std::string::npos || l.find(' ', sp + 1) != std::string::npos) {
            delete t;
            return tok_fail("ce_tokenizer_create: malformed merges line (expected 'a b')");
        }
        t->ranks[l] = rank++;          // later duplicates win, as dict(zip(merges, range()))
        vocab.push_back(l.substr(0, sp) + l.substr(sp + 1));
    }
    t->specials = {"<start_of_text>", "<end_of_text>"};
    for (int k = 0; k < n_extra; ++k)
        if (extra_special && extra_special[k]) t->specials.push_back(extra_special[k]);
    for (const std::string& s : t->specials) vocab.push_back(s);
    t->decoder = vocab;
    for (size_t k = 0; k < vocab.size(); ++k) t->encoder[vocab[k]] = (int32_t)k;   // later entries win, as dict(zip())
    t->sot = t->encoder["<start_of_text>"];
    t->eot = t->encoder["<end_of_text>"];
    *out = t;
    return 0;
}

int ce_tokenizer_destroy(ce_tokenizer* t) {
    delete t;
    return 0;
}

int ce_tokenizer_vocab_size(const ce_tokenizer* t) { return t ? (int)t->encoder.size() : 0; }

int ce_tokenizer_special_ids(const ce_tokenizer* t, int32_t* sot, int32_t* eot) {
    if (!t) return tok_fail("ce_tokenizer_special_ids: null tokenizer");
    if (sot) *sot = t->sot;
    if (eot) *eot = t->eot;
    return 0;
}

int ce_tokenizer_encode(ce_tokenizer* t, const char* text, int32_t* ids, int cap, int* n_out) {
    if (!t || !text || !n_out) return tok_fail("ce_tokenizer_encode: null argument");
    std::vector<int32_t> v;
    t->encode(text, v);
    *n_out = (int)v.size();
    if (ids) memcpy(ids, v.data(), sizeof(int32_t) * std::min<size_t>(v.size(), cap > 0 ? (size_t)cap : 0));
    return 0;
}

int ce_tokenize(ce_tokenizer* t, const char* const* texts, int n, int context_length, int64_t* out) {
    if (!t || (!texts && n > 0) || (!out && n > 0)) return tok_fail("ce_tokenize: null argument");
    if (context_length <= 0) return tok_fail("ce_tokenize: context_length must be positive");
    std::vector<int32_t> v;
    for (int i = 0; i < n; ++i) {
        v.clear();
        v.push_back(t->sot);
        if (texts[i]) t->encode(texts[i], v);
        v.push_back(t->eot);
        if ((int)v.size() > context_length) {
            v.resize(context_length);
            v.back() = t->eot;
        }
        int64_t* row = out + (size_t)i * context_length;
        for (int k = 0; k < context_length; ++k) row[k] = k < (int)v.size() ? v[k] : 0;
    }
    return 0;
}

// decode (tokenizer.py:221-224): concatenated symbols -> bytes -> UTF-8 ("</w>" -> " ").  Bytes that
// are not valid UTF-8 become U+FFFD (Python's errors="replace" for the common cases).
int ce_tokenizer_decode(const ce_tokenizer* t, const int32_t* ids, int n, char* buf, int cap, int* len_out) {
    if (!t || (!ids && n > 0) || !len_out) return tok_fail("ce_tokenizer_decode: null argument");
    std::string sym;
    for (int i = 0; i < n; ++i) {
        if (ids[i] < 0 || ids[i] >= (int32_t)t->decoder.size()) return tok_fail("ce_tokenizer_decode: id out of range");
        sym += t->decoder[ids[i]];
    }
    std::string bytes;
    for (size_t i = 0; i < sym.size();) {     // "</w>" is four printable byte symbols: kept as text
        uint32_t cp;
        const int k = next_cp(sym, i, cp);
        auto it = t->sym_byte.find(cp);
        if (it != t->sym_byte.end()) bytes += (char)it->second;
        i += k;
    }
    std::string txt;
    for (size_t i = 0; i < bytes.size();) {
        const unsigned char c = (unsigned char)bytes[i];
        int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        bool ok = len > 0 && i + len <= bytes.size();
        for (int k = 1; ok && k < len; ++k) ok = ((unsigned char)bytes[i + k] >> 6) == 2;
        if (ok) {
            txt.append(bytes, i, len);
            i += len;
        } else {
            put_utf8(txt, 0xFFFD);
            i += 1;
        }
    }
    std::string res;
    for (size_t i = 0; i < txt.size();) {
        if (txt.compare(i, 4, "</w>") == 0) {
            res += ' ';
            i += 4;
        } else {
            res += txt[i++];
        }
    }
    *len_out = (int)res.size();
    if (buf && cap > 0) {
        const size_t m = std::min<size_t>(res.size(), (size_t)cap - 1);
        memcpy(buf, res.data(), m);
        buf[m] = 0;
    }
    return 0;
}

}  // extern "C"
