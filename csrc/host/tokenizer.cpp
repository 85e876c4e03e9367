// See tokenizer.h.
#include "tokenizer.h"

#include <pybind11/stl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <limits>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace ragtl {
namespace {

// ---------------------------------------------------------------- UTF-8 helpers
std::vector<std::string> utf8_chars(const std::string& s) {
  std::vector<std::string> out;
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
    if (i + n > s.size()) n = 1;
    out.emplace_back(s.substr(i, n));
    i += n;
  }
  return out;
}

std::string cp_to_utf8(uint32_t cp) {
  std::string o;
  if (cp < 0x80) o.push_back((char)cp);
  else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) {
    o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    o.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F)));
  }
  return o;
}

bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }
bool is_ascii_punct(unsigned char c) {
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}
bool is_alpha(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c >= 0x80; }
bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

// GPT-2 byte <-> unicode map
struct ByteMap {
  std::string enc[256];
  std::unordered_map<std::string, int> dec;
  ByteMap() {
    std::vector<int> bs;
    for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
    for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
    for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
    std::vector<int> cs = bs;
    int n = 0;
    for (int b = 0; b < 256; ++b)
      if (std::find(bs.begin(), bs.end(), b) == bs.end()) { bs.push_back(b); cs.push_back(256 + n); ++n; }
    for (size_t i = 0; i < bs.size(); ++i) {
      enc[bs[i]] = cp_to_utf8((uint32_t)cs[i]);
      dec[enc[bs[i]]] = bs[i];
    }
  }
};
const ByteMap& bytemap() {
  static ByteMap m;
  return m;
}

struct PairHash {
  size_t operator()(const std::pair<std::string, std::string>& p) const {
    return std::hash<std::string>()(p.first) * 1000003u ^ std::hash<std::string>()(p.second);
  }
};

}  // namespace

class Tokenizer {
 public:
  // kind: "wordlevel" | "wordpiece" | "bpe" (byte-level) | "sp_bpe" (metaspace + byte fallback)
  Tokenizer(std::string kind, std::unordered_map<std::string, int64_t> vocab,
            std::vector<std::pair<std::string, std::string>> merges, std::string unk_token, bool lowercase,
            std::string continuing_prefix, bool add_prefix_space, bool byte_fallback,
            std::vector<std::string> special_tokens)
      : kind_(std::move(kind)), vocab_(std::move(vocab)), unk_(std::move(unk_token)), lower_(lowercase),
        cont_(std::move(continuing_prefix)), prefix_space_(add_prefix_space), byte_fallback_(byte_fallback) {
    int64_t maxid = -1;
    for (auto& kv : vocab_) maxid = std::max(maxid, kv.second);
    inv_.assign(maxid + 1, "");
    for (auto& kv : vocab_) inv_[kv.second] = kv.first;
    for (size_t i = 0; i < merges.size(); ++i) ranks_[merges[i]] = (int)i;
    for (auto& s : special_tokens) specials_[s] = vocab_.count(s) ? vocab_[s] : -1;
    auto it = vocab_.find(unk_);
    unk_id_ = it == vocab_.end() ? -1 : it->second;
  }

  std::vector<int64_t> encode(const std::string& text) const {
    std::vector<int64_t> out;
    // split out special tokens verbatim
    size_t i = 0;
    std::string chunk;
    while (i < text.size()) {
      bool matched = false;
      for (auto& sp : specials_) {
        if (sp.second >= 0 && !sp.first.empty() && text.compare(i, sp.first.size(), sp.first) == 0) {
          if (!chunk.empty()) { encode_chunk(chunk, out); chunk.clear(); }
          out.push_back(sp.second);
          i += sp.first.size();
          matched = true;
          break;
        }
      }
      if (!matched) chunk.push_back(text[i++]);
    }
    if (!chunk.empty()) encode_chunk(chunk, out);
    return out;
  }

  std::vector<std::vector<int64_t>> encode_batch(const std::vector<std::string>& texts, int nthreads) const {
    std::vector<std::vector<int64_t>> out(texts.size());
    if (nthreads <= 1 || texts.size() < 64) {
      for (size_t i = 0; i < texts.size(); ++i) out[i] = encode(texts[i]);
      return out;
    }
    py::gil_scoped_release release;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([&, t] {
        for (size_t i = t; i < texts.size(); i += nthreads) out[i] = encode(texts[i]);
      });
    for (auto& x : th) x.join();
    return out;
  }

  std::string decode(const std::vector<int64_t>& ids, bool skip_special) const {
    std::string o;
    std::string bytes_pending;
    bool first = true;
    for (int64_t id : ids) {
      if (id < 0 || id >= (int64_t)inv_.size()) continue;
      const std::string& tok = inv_[id];
      if (skip_special && specials_.count(tok)) continue;
      if (kind_ == "bpe") {
        for (auto& ch : utf8_chars(tok)) {
          auto it = bytemap().dec.find(ch);
          if (it != bytemap().dec.end()) o.push_back((char)it->second);
          else o += ch;
        }
      } else if (kind_ == "sp_bpe") {
        if (byte_fallback_ && tok.size() == 6 && tok[0] == '<' && tok[1] == '0' && tok[2] == 'x' && tok[5] == '>') {
          o.push_back((char)std::stoi(tok.substr(3, 2), nullptr, 16));
          continue;
        }
        std::string t = tok;
        std::string r;
        for (auto& ch : utf8_chars(t)) r += (ch == "\xE2\x96\x81") ? std::string(" ") : ch;
        o += r;
      } else if (kind_ == "wordpiece") {
        if (!cont_.empty() && tok.compare(0, cont_.size(), cont_) == 0) o += tok.substr(cont_.size());
        else { if (!first) o.push_back(' '); o += tok; }
      } else {
        if (!first) o.push_back(' ');
        o += tok;
      }
      first = false;
    }
    if (kind_ == "sp_bpe" && prefix_space_ && !o.empty() && o[0] == ' ') o.erase(0, 1);
    return o;
  }

  int64_t token_to_id(const std::string& t) const {
    auto it = vocab_.find(t);
    return it == vocab_.end() ? -1 : it->second;
  }
  std::string id_to_token(int64_t id) const { return (id >= 0 && id < (int64_t)inv_.size()) ? inv_[id] : ""; }
  int64_t vocab_size() const { return (int64_t)inv_.size(); }

 private:
  void push_word(const std::string& w, std::vector<int64_t>& out) const {
    auto it = vocab_.find(w);
    if (it != vocab_.end()) out.push_back(it->second);
    else if (unk_id_ >= 0) out.push_back(unk_id_);
  }

  // basic pre-tokenisation: whitespace split, punctuation isolated (BERT BasicTokenizer, ASCII)
  std::vector<std::string> basic_split(const std::string& s) const {
    std::vector<std::string> words;
    std::string cur;
    for (unsigned char c : s) {
      if (is_space(c)) { if (!cur.empty()) { words.push_back(cur); cur.clear(); } continue; }
      if (is_ascii_punct(c)) {
        if (!cur.empty()) { words.push_back(cur); cur.clear(); }
        words.push_back(std::string(1, (char)c));
        continue;
      }
      cur.push_back(lower_ && c < 0x80 ? (char)std::tolower(c) : (char)c);
    }
    if (!cur.empty()) words.push_back(cur);
    return words;
  }

  void wordpiece(const std::string& word, std::vector<int64_t>& out) const {
    auto chars = utf8_chars(word);
    if (chars.size() > 100) { if (unk_id_ >= 0) out.push_back(unk_id_); return; }
    std::vector<int64_t> pieces;
    size_t start = 0;
    while (start < chars.size()) {
      size_t end = chars.size();
      int64_t found = -1;
      while (start < end) {
        std::string sub;
        for (size_t k = start; k < end; ++k) sub += chars[k];
        if (start > 0) sub = cont_ + sub;
        auto it = vocab_.find(sub);
        if (it != vocab_.end()) { found = it->second; break; }
        --end;
      }
      if (found < 0) { if (unk_id_ >= 0) out.push_back(unk_id_); return; }
      pieces.push_back(found);
      start = end;
    }
    out.insert(out.end(), pieces.begin(), pieces.end());
  }

  std::vector<std::string> bpe_merge(std::vector<std::string> sym) const {
    while (sym.size() > 1) {
      int best = std::numeric_limits<int>::max();
      size_t bi = 0;
      for (size_t k = 0; k + 1 < sym.size(); ++k) {
        auto it = ranks_.find({sym[k], sym[k + 1]});
        if (it != ranks_.end() && it->second < best) { best = it->second; bi = k; }
      }
      if (best == std::numeric_limits<int>::max()) break;
      std::vector<std::string> nxt;
      nxt.reserve(sym.size());
      const std::string a = sym[bi], b = sym[bi + 1];
      for (size_t k = 0; k < sym.size();) {
        if (k + 1 < sym.size() && sym[k] == a && sym[k + 1] == b) { nxt.push_back(a + b); k += 2; }
        else { nxt.push_back(sym[k]); k += 1; }
      }
      sym.swap(nxt);
    }
    return sym;
  }

  // GPT-2 style pre-tokeniser (ASCII classes; bytes >= 0x80 treated as letters)
  std::vector<std::string> gpt2_split(const std::string& s) const {
    std::vector<std::string> out;
    size_t i = 0, n = s.size();
    auto cls = [](unsigned char c) { return is_alpha(c) ? 1 : is_digit(c) ? 2 : is_space(c) ? 3 : 4; };
    while (i < n) {
      if (s[i] == '\'' && i + 1 < n) {
        static const char* contr[] = {"'s", "'t", "'re", "'ve", "'m", "'ll", "'d"};
        bool hit = false;
        for (auto* c : contr) {
          const size_t L = strlen(c);
          if (s.compare(i, L, c) == 0) { out.push_back(s.substr(i, L)); i += L; hit = true; break; }
        }
        if (hit) continue;
      }
      size_t j = i;
      const bool lead_space = s[i] == ' ' && i + 1 < n && cls((unsigned char)s[i + 1]) != 3;
      if (lead_space) ++j;
      const int c0 = cls((unsigned char)s[j]);
      if (c0 == 3) {
        // \s+(?!\S) | \s+ : run of spaces, leaving the last one for the next word if followed by non-space
        size_t k = j;
        while (k < n && is_space((unsigned char)s[k])) ++k;
        if (k < n && k - j > 1) --k;
        out.push_back(s.substr(i, k - i));
        i = k;
        continue;
      }
      size_t k = j;
      while (k < n && cls((unsigned char)s[k]) == c0) ++k;
      out.push_back(s.substr(i, k - i));
      i = k;
    }
    return out;
  }

  void encode_chunk(const std::string& text, std::vector<int64_t>& out) const {
    if (kind_ == "wordlevel") {
      for (auto& w : basic_split(text)) push_word(w, out);
    } else if (kind_ == "wordpiece") {
      for (auto& w : basic_split(text)) wordpiece(w, out);
    } else if (kind_ == "bpe") {
      std::string t = (prefix_space_ && !text.empty() && text[0] != ' ') ? " " + text : text;
      for (auto& w : gpt2_split(t)) {
        std::vector<std::string> sym;
        for (unsigned char c : w) sym.push_back(bytemap().enc[c]);
        for (auto& p : bpe_merge(sym)) push_word(p, out);
      }
    } else {  // sp_bpe
      std::string t;
      if (prefix_space_) t = "\xE2\x96\x81";
      for (char c : text) t += (c == ' ') ? std::string("\xE2\x96\x81") : std::string(1, c);
      auto syms = bpe_merge(utf8_chars(t));
      for (auto& p : syms) {
        auto it = vocab_.find(p);
        if (it != vocab_.end()) { out.push_back(it->second); continue; }
        if (byte_fallback_) {
          for (unsigned char c : p) {
            char buf[8];
            snprintf(buf, sizeof(buf), "<0x%02X>", c);
            auto bt = vocab_.find(buf);
            if (bt != vocab_.end()) out.push_back(bt->second);
            else if (unk_id_ >= 0) out.push_back(unk_id_);
          }
        } else if (unk_id_ >= 0) {
          out.push_back(unk_id_);
        }
      }
    }
  }

  std::string kind_;
  std::unordered_map<std::string, int64_t> vocab_;
  std::vector<std::string> inv_;
  std::unordered_map<std::pair<std::string, std::string>, int, PairHash> ranks_;
  std::unordered_map<std::string, int64_t> specials_;
  std::string unk_;
  int64_t unk_id_;
  bool lower_;
  std::string cont_;
  bool prefix_space_;
  bool byte_fallback_;
};

void bind_tokenizer(py::module& m) {
  py::class_<Tokenizer>(m, "NativeTokenizer")
      .def(py::init<std::string, std::unordered_map<std::string, int64_t>,
                    std::vector<std::pair<std::string, std::string>>, std::string, bool, std::string, bool, bool,
                    std::vector<std::string>>(),
           py::arg("kind"), py::arg("vocab"), py::arg("merges"), py::arg("unk_token"), py::arg("lowercase"),
           py::arg("continuing_prefix"), py::arg("add_prefix_space"), py::arg("byte_fallback"),
           py::arg("special_tokens"))
      .def("encode", &Tokenizer::encode)
      .def("encode_batch", &Tokenizer::encode_batch, py::arg("texts"), py::arg("nthreads") = 8)
      .def("decode", &Tokenizer::decode, py::arg("ids"), py::arg("skip_special") = true)
      .def("token_to_id", &Tokenizer::token_to_id)
      .def("id_to_token", &Tokenizer::id_to_token)
      .def("vocab_size", &Tokenizer::vocab_size);
}

}  // namespace ragtl
