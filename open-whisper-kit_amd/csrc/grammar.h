// GBNF grammar parse state of one decoder (ref src/whisper.cpp:769-781, 5498-5905); grammar.cpp.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "whisper.h"

namespace owk {

struct GPos {  // element `elem` of rule `rule`
    int rule = 0, elem = 0;
};
using Stack = std::vector<GPos>;

struct Partial {  // trailing incomplete UTF-8 sequence (ref whisper_partial_utf8)
    uint32_t value = 0;
    int n_remain = 0;
};

struct Grammar {
    std::shared_ptr<const std::vector<std::vector<whisper_grammar_element>>> rules;  // immutable, shared by copies
    std::vector<Stack> stacks;
    Partial partial;

    // whisper_grammar_init (ref 5771-5808); no rules (null / 0) leaves the grammar inactive
    void init(const whisper_grammar_element ** rules, size_t n_rules, size_t i_start_rule);
    // whisper_suppress_invalid_grammar (ref 5810-5855): logits[id] -= penalty for every text token
    // (id < eot, non-empty text) no stack can accept
    void suppress(const std::vector<std::string> & id_to_token, int eot, float penalty, float * logits) const;
    // whisper_grammar_accept_token (ref 5857-5880) for the token's text
    void accept(const std::string & token_text);
    bool active() const { return rules && !rules->empty(); }
};

} // namespace owk
