// Sanitizer harness for the host BPE core (csrc/host/bpe_core.h): built with
// -fsanitize=address,undefined by tests/test_native_sanitizers.py and run on random byte strings
// (valid UTF-8 of every width, truncated / invalid sequences, contractions, digit runs, mixed
// whitespace and newlines) under both pre-tokenisers.  Checks, besides "no sanitizer report":
//   * pre_tokenize pieces tile the input exactly (contiguous, non-empty, cover every byte);
//   * encode_ordinary ids decode back to the input bytes (vocabulary inverse map).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../csrc/host/bpe_core.h"

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  std::mt19937 rng(1234);
  // vocabulary: all 256 bytes + a few hundred random merges of existing tokens
  std::unordered_map<std::string, int> ranks;
  std::vector<std::string> toks;
  for (int b = 0; b < 256; ++b) {
    toks.emplace_back(1, (char)b);
    ranks.emplace(toks.back(), b);
  }
  const char* common[] = {"th", "he", "in", "er", "an", " t", " a", "the", " the", "ing", "'s", "12", "  ", "\n\n"};
  for (const char* c : common)
    if (!ranks.count(c)) { ranks.emplace(c, (int)toks.size()); toks.emplace_back(c); }
  for (int i = 0; i < 400; ++i) {
    std::string t = toks[rng() % toks.size()] + toks[rng() % toks.size()];
    if (!ranks.count(t)) { ranks.emplace(t, (int)toks.size()); toks.push_back(t); }
  }
  // class table for code points < 0x3000: letters / numbers / whitespace / other (ASCII-exact)
  std::string classes(0x3000, (char)1);
  for (int c = 0; c < 128; ++c) {
    char k = 0;
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) k = 1;
    else if (c >= '0' && c <= '9') k = 2;
    else if (c == ' ' || (c >= 9 && c <= 13)) k = 3;
    classes[c] = k;
  }
  const char* frags[] = {"the ", "The", "'s", "'LL", "'ve", " 123", "4567", "\r\n", "\n\n\n", "   ", "\t",
                         "!?", "...", "\xc3\xa9", "\xe4\xb8\xad", "\xf0\x9f\x98\x80", "\xe4", "\xf0\x9f", "\xff",
                         "x", " y", "\x80\x80"};
  const int nfr = sizeof(frags) / sizeof(frags[0]);
  for (const char* kind : {"gpt2", "llama3"}) {
    bllm_host::BPECore core(ranks, kind, classes);
    for (int it = 0; it < iters; ++it) {
      std::string s;
      const int n = rng() % 40;
      for (int k = 0; k < n; ++k) {
        if (rng() % 4 == 0) s.push_back((char)(rng() & 0xFF));
        else s += frags[rng() % nfr];
      }
      size_t pos = 0;
      for (auto& pr : core.pre_tokenize(s)) {
        if (pr.first != pos || pr.second <= pr.first) { std::printf("FAIL tiling %s\n", kind); return 1; }
        pos = pr.second;
      }
      if (pos != s.size()) { std::printf("FAIL cover %s\n", kind); return 1; }
      std::string back;
      for (int id : core.encode_ordinary(s)) back += toks[id];
      if (back != s) { std::printf("FAIL roundtrip %s\n", kind); return 1; }
    }
  }
  std::printf("bpe_fuzz ok (%d iterations x 2 pre-tokenisers)\n", iters);
  return 0;
}
