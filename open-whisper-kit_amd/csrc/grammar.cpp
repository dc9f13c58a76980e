// GBNF grammar-constrained decoding on the host logits path (ref src/whisper.cpp:5498-5905, used at
// 6363-6384, 7113-7117, 7263, 7334, 7391).
//
// The grammar is a set of rules, each a sequence of whisper_grammar_element alternatives; a parse
// state is a set of pushdown stacks whose tops all sit on a character class. Positions are held as
// (rule, element) indices, so a state copies freely between decoders (beam search) -- the
// reference keeps raw element pointers; both address the same immutable rule text.
//   * whisper_grammar_init: expand every alternative of the start rule to character-class tops;
//   * suppress (per decode step, only where the timestamp-mass rule left text tokens): every text
//     token whose UTF-8 bytes no stack can consume (given the partial code point carried from the
//     previous token) gets grammar_penalty subtracted from its logit;
//   * accept (per sampled token, "[_" special tokens skipped): advance every stack over the
//     token's code points, keep the trailing partial UTF-8 sequence.
#include "grammar.h"

#include <algorithm>

namespace owk {

namespace {

using Rules = std::vector<std::vector<whisper_grammar_element>>;

struct Utf8 {
    std::vector<uint32_t> cps;  // code points, terminated by 0
    Partial partial;
};

// UTF-8 bytes of a NUL-terminated string, continuing `start` (ref decode_utf8, 5498-5551): an
// invalid byte ends the sequence with code point 0 and n_remain -1
Utf8 decode(const char * s, Partial start) {
    static const int len_of_hi[16] = {1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 2, 2, 3, 4};
    Utf8 r;
    const unsigned char * p = (const unsigned char *) s;
    uint32_t value = start.value;
    int rem = start.n_remain;
    while (*p && rem > 0) {
        if ((*p >> 6) != 2) {  // not a continuation byte
            r.cps.push_back(0);
            r.partial = {0, -1};
            return r;
        }
        value = (value << 6) + (*p & 0x3F);
        ++p;
        --rem;
    }
    if (start.n_remain > 0 && rem == 0) r.cps.push_back(value);
    while (*p) {
        rem = len_of_hi[*p >> 4] - 1;
        if (rem < 0) {
            r.cps.assign(1, 0);
            r.partial = {0, rem};
            return r;
        }
        value = *p & ((1u << (7 - rem)) - 1);
        ++p;
        while (*p && rem > 0) {
            value = (value << 6) + (*p & 0x3F);
            ++p;
            --rem;
        }
        if (rem == 0) r.cps.push_back(value);
    }
    r.cps.push_back(0);
    r.partial = {value, rem};
    return r;
}

const whisper_grammar_element & el(const Rules & R, GPos p) { return R[p.rule][p.elem]; }

bool ends_alternative(const Rules & R, GPos p) {
    const auto t = el(R, p).type;
    return t == WHISPER_GRETYPE_END || t == WHISPER_GRETYPE_ALT;
}

// does code point c satisfy the character class at p? also returns the element after the class
// (ref whisper_grammar_match_char, 5562-5587)
bool match_char(const Rules & R, GPos p, uint32_t c, GPos & after) {
    const bool positive = el(R, p).type == WHISPER_GRETYPE_CHAR;
    bool hit = false;
    do {
        const GPos nx{p.rule, p.elem + 1};
        if (el(R, nx).type == WHISPER_GRETYPE_CHAR_RNG_UPPER) {
            hit = hit || (el(R, p).value <= c && c <= el(R, nx).value);
            p.elem += 2;
        } else {
            hit = hit || el(R, p).value == c;
            p.elem += 1;
        }
    } while (el(R, p).type == WHISPER_GRETYPE_CHAR_ALT);
    after = p;
    return hit == positive;
}

// can some completion of the partial sequence satisfy the class at p? (ref 5591-5634)
bool match_partial(const Rules & R, GPos p, Partial part) {
    const bool positive = el(R, p).type == WHISPER_GRETYPE_CHAR;
    const int rem = part.n_remain;
    if (rem < 0 || (rem == 1 && part.value < 2)) return false;  // invalid or overlong
    uint32_t lo = part.value << (rem * 6);
    const uint32_t hi = lo | ((1u << (rem * 6)) - 1);
    if (lo == 0) {
        if (rem == 2) lo = 1u << 11;
        else if (rem == 3) lo = 1u << 16;
    }
    do {
        const GPos nx{p.rule, p.elem + 1};
        if (el(R, nx).type == WHISPER_GRETYPE_CHAR_RNG_UPPER) {
            if (el(R, p).value <= hi && lo <= el(R, nx).value) return positive;
            p.elem += 2;
        } else {
            if (lo <= el(R, p).value && el(R, p).value <= hi) return positive;
            p.elem += 1;
        }
    } while (el(R, p).type == WHISPER_GRETYPE_CHAR_ALT);
    return !positive;
}

// expand the top of `stack` until every resulting stack's top is a character class (or the stack
// is empty), appending them to `out` in the reference's order (ref whisper_grammar_advance_stack)
void expand(const Rules & R, const Stack & stack, std::vector<Stack> & out) {
    if (stack.empty()) {
        out.emplace_back();
        return;
    }
    const GPos top = stack.back();
    const auto & e = el(R, top);
    if (e.type == WHISPER_GRETYPE_CHAR || e.type == WHISPER_GRETYPE_CHAR_NOT) {
        out.push_back(stack);
        return;
    }
    if (e.type != WHISPER_GRETYPE_RULE_REF) throw std::runtime_error("grammar: stack top is not a rule or a class");
    const int rule = (int) e.value;
    if (rule < 0 || rule >= (int) R.size()) throw std::runtime_error("grammar: rule reference out of range");
    GPos alt{rule, 0};
    for (;;) {
        Stack ns(stack.begin(), stack.end() - 1);
        const GPos next{top.rule, top.elem + 1};
        if (!ends_alternative(R, next)) ns.push_back(next);
        if (!ends_alternative(R, alt)) ns.push_back(alt);
        expand(R, ns, out);
        while (!ends_alternative(R, alt)) alt.elem++;
        if (el(R, alt).type != WHISPER_GRETYPE_ALT) break;
        alt.elem++;
    }
}

// the stacks after consuming code point c (ref whisper_grammar_accept)
std::vector<Stack> consume(const Rules & R, const std::vector<Stack> & stacks, uint32_t c) {
    std::vector<Stack> out;
    for (const Stack & s : stacks) {
        if (s.empty()) continue;
        GPos after;
        if (!match_char(R, s.back(), c, after)) continue;
        Stack ns(s.begin(), s.end() - 1);
        if (!ends_alternative(R, after)) ns.push_back(after);
        expand(R, ns, out);
    }
    return out;
}

struct Cand {
    int id;
    const uint32_t * cp;  // next code point of the token's decoded text
    Partial partial;
};

std::vector<Cand> reject(const Rules & R, const std::vector<Stack> & stacks, const std::vector<Cand> & cands);

// candidates that the single stack `s` cannot accept (ref 5686-5736)
std::vector<Cand> reject_one(const Rules & R, const Stack & s, const std::vector<Cand> & cands) {
    std::vector<Cand> rej;
    if (s.empty()) {
        for (const Cand & c : cands)
            if (*c.cp != 0 || c.partial.n_remain != 0) rej.push_back(c);
        return rej;
    }
    const GPos top = s.back();
    std::vector<Cand> next;
    for (const Cand & c : cands) {
        GPos unused;
        if (*c.cp == 0) {
            if (c.partial.n_remain != 0 && !match_partial(R, top, c.partial)) rej.push_back(c);
        } else if (match_char(R, top, *c.cp, unused)) {
            next.push_back({c.id, c.cp + 1, c.partial});
        } else {
            rej.push_back(c);
        }
    }
    GPos after;
    match_char(R, top, 0, after);
    Stack ns(s.begin(), s.end() - 1);
    if (!ends_alternative(R, after)) ns.push_back(after);
    std::vector<Stack> nstacks;
    expand(R, ns, nstacks);
    for (const Cand & c : reject(R, nstacks, next)) rej.push_back({c.id, c.cp - 1, c.partial});
    return rej;
}

// candidates no stack accepts: rejected by the first stack, then re-tested against each further one
std::vector<Cand> reject(const Rules & R, const std::vector<Stack> & stacks, const std::vector<Cand> & cands) {
    if (cands.empty() || stacks.empty()) return {};
    std::vector<Cand> rej = reject_one(R, stacks.front(), cands);
    for (size_t i = 1; i < stacks.size(); ++i) rej = reject_one(R, stacks[i], rej);
    return rej;
}

} // namespace

void Grammar::init(const whisper_grammar_element ** rules_in, size_t n_rules, size_t i_start) {
    rules.reset();
    stacks.clear();
    partial = Partial{};
    if (!rules_in || n_rules == 0) return;
    if (i_start >= n_rules) throw std::runtime_error("grammar: start rule out of range");
    auto R = std::make_shared<Rules>(n_rules);
    for (size_t i = 0; i < n_rules; ++i) {
        for (const whisper_grammar_element * p = rules_in[i]; p->type != WHISPER_GRETYPE_END; ++p) (*R)[i].push_back(*p);
        (*R)[i].push_back({WHISPER_GRETYPE_END, 0});
    }
    GPos alt{(int) i_start, 0};
    for (;;) {
        Stack s;
        if (!ends_alternative(*R, alt)) s.push_back(alt);
        expand(*R, s, stacks);
        while (!ends_alternative(*R, alt)) alt.elem++;
        if (el(*R, alt).type != WHISPER_GRETYPE_ALT) break;
        alt.elem++;
    }
    rules = std::move(R);
}

void Grammar::suppress(const std::vector<std::string> & id_to_token, int eot, float penalty, float * logits) const {
    if (!rules || rules->empty() || stacks.empty()) return;
    std::vector<Utf8> dec;
    std::vector<int> ids;
    dec.reserve(eot);
    for (int id = 0; id < eot; ++id) {
        const std::string & t = id_to_token[id];
        if (t.empty()) continue;
        dec.push_back(decode(t.c_str(), partial));
        ids.push_back(id);
    }
    std::vector<Cand> cands(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) cands[i] = {ids[i], dec[i].cps.data(), dec[i].partial};
    for (const Cand & c : reject(*rules, stacks, cands)) logits[c.id] -= penalty;
}

void Grammar::accept(const std::string & text) {
    if (!rules || rules->empty() || stacks.empty()) return;
    if (text.rfind("[_", 0) == 0) return;  // timestamp / special token text
    const Utf8 d = decode(text.c_str(), partial);
    for (size_t i = 0; i + 1 < d.cps.size(); ++i) stacks = consume(*rules, stacks, d.cps[i]);
    partial = d.partial;
}

} // namespace owk
