// Byte-level BPE core (pre-tokenisation + rank merging), free of Python: bound by bpe.cpp
// (pybind11 module ``_bpe``) and exercised under AddressSanitizer / UBSan by bpe_fuzz.cpp
// (tests/test_native_sanitizers.py).  See bpe.cpp for the algorithm notes.
#pragma once
#include <cstdint>
#include <climits>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace bllm_host {

enum : uint8_t { C_OTHER = 0, C_LETTER = 1, C_NUMBER = 2, C_SPACE = 3 };

struct Piece {
  size_t b0, b1;  // byte range in the UTF-8 text
};

class BPECore {
 public:
  BPECore(std::unordered_map<std::string, int> ranks, const std::string& kind, const std::string& classes)
      : ranks_(std::move(ranks)) {
    if (kind == "gpt2") kind_ = 0;
    else if (kind == "llama3") kind_ = 1;
    else throw std::invalid_argument("BPECore: kind must be 'gpt2' or 'llama3'");
    cls_.assign(classes.begin(), classes.end());
  }

  std::vector<int> encode_ordinary(const std::string& text) {
    decode_utf8(text);
    std::vector<Piece> pieces;
    if (kind_ == 0) split_gpt2(pieces); else split_llama3(pieces);
    std::vector<int> out;
    out.reserve(text.size() / 3 + 4);
    for (const Piece& p : pieces) bpe(text.data() + p.b0, p.b1 - p.b0, out);
    return out;
  }

  std::vector<std::pair<size_t, size_t>> pre_tokenize(const std::string& text) {
    decode_utf8(text);
    std::vector<Piece> pieces;
    if (kind_ == 0) split_gpt2(pieces); else split_llama3(pieces);
    std::vector<std::pair<size_t, size_t>> r;
    for (auto& p : pieces) r.emplace_back(p.b0, p.b1);
    return r;
  }

  size_t cache_size() const { return cache_.size(); }

 private:
  std::unordered_map<std::string, int> ranks_;
  std::unordered_map<std::string, std::vector<int>> cache_;
  std::vector<uint8_t> cls_;
  int kind_ = 0;
  // decoded text
  std::vector<uint32_t> cp_;
  std::vector<size_t> off_;  // byte offset of each code point (+ sentinel)

  void decode_utf8(const std::string& s) {
    cp_.clear();
    off_.clear();
    const auto* b = reinterpret_cast<const unsigned char*>(s.data());
    const size_t n = s.size();
    size_t i = 0;
    while (i < n) {
      uint32_t c = b[i];
      size_t len = 1;
      if ((c >> 5) == 0x6) len = 2;
      else if ((c >> 4) == 0xE) len = 3;
      else if ((c >> 3) == 0x1E) len = 4;
      if (i + len > n) len = n - i;  // truncated sequence: consume the rest as one unit
      if (len == 2) c = ((c & 0x1F) << 6) | (b[i + 1] & 0x3F);
      else if (len == 3) c = ((c & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F);
      else if (len == 4)
        c = ((c & 0x07) << 18) | ((b[i + 1] & 0x3F) << 12) | ((b[i + 2] & 0x3F) << 6) | (b[i + 3] & 0x3F);
      cp_.push_back(c);
      off_.push_back(i);
      i += len;
    }
    off_.push_back(n);
  }

  uint8_t cls(size_t i) const {
    const uint32_t c = cp_[i];
    return c < cls_.size() ? cls_[c] : C_LETTER;  // beyond the table: supplementary ideographs etc.
  }
  bool is_letter(size_t i) const { return cls(i) == C_LETTER; }
  bool is_number(size_t i) const { return cls(i) == C_NUMBER; }
  bool is_space(size_t i) const { return cls(i) == C_SPACE; }
  bool is_other(size_t i) const { return cls(i) == C_OTHER; }  // [^\s\p{L}\p{N}]
  bool is_nl(size_t i) const { return cp_[i] == '\r' || cp_[i] == '\n'; }

  static uint32_t lower(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

  // contraction 's 't 're 've 'm 'll 'd starting at i (apostrophe at i); returns length or 0
  size_t contraction(size_t i, bool icase) const {
    const size_t n = cp_.size();
    if (cp_[i] != '\'' || i + 1 >= n) return 0;
    auto ch = [&](size_t k) -> uint32_t { return icase ? lower(cp_[k]) : cp_[k]; };
    const uint32_t a = ch(i + 1);
    if (a == 's' || a == 't' || a == 'm' || a == 'd') return 2;
    if (i + 2 < n) {
      const uint32_t b = ch(i + 2);
      if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return 3;
    }
    return 0;
  }

  // \s+(?!\S) then \s+ : maximal whitespace run [i, j); if followed by a non-space and the run
  // is longer than one, leave the last whitespace for the next token
  size_t whitespace(size_t i) const {
    const size_t n = cp_.size();
    size_t j = i;
    while (j < n && is_space(j)) ++j;
    if (j < n && j - i > 1) return j - i - 1;
    return j - i;
  }

  void split_gpt2(std::vector<Piece>& out) const {
    const size_t n = cp_.size();
    size_t i = 0;
    while (i < n) {
      size_t len = contraction(i, false);
      if (!len) {
        const size_t s = (cp_[i] == ' ' && i + 1 < n) ? 1 : 0;  // optional leading space
        size_t j = i + s;
        if (j < n && is_letter(j)) {
          while (j < n && is_letter(j)) ++j;
          len = j - i;
        } else if (j < n && is_number(j)) {
          while (j < n && is_number(j)) ++j;
          len = j - i;
        } else if (j < n && is_other(j)) {
          while (j < n && is_other(j)) ++j;
          len = j - i;
        }
      }
      if (!len) {
        if (is_space(i)) len = whitespace(i);
        else len = 1;  // defensive: every code point is in exactly one class
      }
      out.push_back({off_[i], off_[i + len]});
      i += len;
    }
  }

  void split_llama3(std::vector<Piece>& out) const {
    const size_t n = cp_.size();
    size_t i = 0;
    while (i < n) {
      size_t len = contraction(i, true);
      // [^\r\n\p{L}\p{N}]?\p{L}+
      if (!len) {
        size_t j = i;
        if (!is_letter(j) && !is_number(j) && !is_nl(j) && j + 1 < n && is_letter(j + 1)) ++j;
        if (is_letter(j)) {
          while (j < n && is_letter(j)) ++j;
          len = j - i;
        }
      }
      // \p{N}{1,3}
      if (!len && is_number(i)) {
        size_t j = i;
        while (j < n && j - i < 3 && is_number(j)) ++j;
        len = j - i;
      }
      //  ?[^\s\p{L}\p{N}]+[\r\n]*
      if (!len) {
        const size_t s = (cp_[i] == ' ' && i + 1 < n && is_other(i + 1)) ? 1 : 0;
        size_t j = i + s;
        if (is_other(j)) {
          while (j < n && is_other(j)) ++j;
          while (j < n && is_nl(j)) ++j;
          len = j - i;
        }
      }
      if (!len && is_space(i)) {
        // \s*[\r\n]+ : the whitespace run up to and including the newline run that holds the
        // run's last newline
        size_t j = i;
        while (j < n && is_space(j)) ++j;
        size_t last_nl = SIZE_MAX;
        for (size_t k = j; k > i; --k)
          if (is_nl(k - 1)) { last_nl = k - 1; break; }
        if (last_nl != SIZE_MAX) {
          size_t e = last_nl + 1;
          while (e < n && is_nl(e)) ++e;
          len = e - i;
        } else {
          len = whitespace(i);
        }
      }
      if (!len) len = 1;
      out.push_back({off_[i], off_[i + len]});
      i += len;
    }
  }

  void bpe(const char* p, size_t n, std::vector<int>& out) {
    std::string key(p, n);
    auto hit = ranks_.find(key);
    if (hit != ranks_.end()) {
      out.push_back(hit->second);
      return;
    }
    auto c = cache_.find(key);
    if (c != cache_.end()) {
      out.insert(out.end(), c->second.begin(), c->second.end());
      return;
    }
    // parts as [start, end) byte ranges; merge the lowest-ranked adjacent pair until none
    std::vector<size_t> bnd(n + 1);
    for (size_t k = 0; k <= n; ++k) bnd[k] = k;
    std::string tmp;
    while (bnd.size() > 2) {
      int best = INT32_MAX;
      size_t bi = 0;
      for (size_t k = 0; k + 2 < bnd.size(); ++k) {
        tmp.assign(p + bnd[k], bnd[k + 2] - bnd[k]);
        auto it = ranks_.find(tmp);
        if (it != ranks_.end() && it->second < best) {
          best = it->second;
          bi = k;
        }
      }
      if (best == INT32_MAX) break;
      bnd.erase(bnd.begin() + bi + 1);
    }
    std::vector<int> ids;
    ids.reserve(bnd.size() - 1);
    for (size_t k = 0; k + 1 < bnd.size(); ++k) {
      tmp.assign(p + bnd[k], bnd[k + 1] - bnd[k]);
      auto it = ranks_.find(tmp);
      if (it == ranks_.end()) throw std::runtime_error("BPECore: byte not in vocabulary");
      ids.push_back(it->second);
    }
    if (cache_.size() < 500000) cache_.emplace(std::move(key), ids);
    out.insert(out.end(), ids.begin(), ids.end());
  }
};

}  // namespace bllm_host

