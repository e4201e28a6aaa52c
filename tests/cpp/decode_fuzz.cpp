// decode_fuzz.cpp -- host sanitizer run of the native history decoder (tests/test_sanitizers.py).
//
// Reads a corpus of valid persisted-history blobs (length-prefixed, written by the test), decodes
// them once intact (must succeed), then decodes thousands of mutated copies -- truncations, flipped
// bytes, corrupted lengths and type bytes -- under AddressSanitizer / UBSan: every call must either
// succeed or return a CRR_DECODE_* error, never read out of bounds or crash.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "cadence_decode.h"

static std::vector<std::vector<uint8_t>> load(const char* path) {
  std::vector<std::vector<uint8_t>> out;
  FILE* f = std::fopen(path, "rb");
  if (!f) return out;
  uint32_t n = 0;
  while (std::fread(&n, 4, 1, f) == 1) {
    std::vector<uint8_t> b(n);
    if (n && std::fread(b.data(), 1, n, f) != n) break;
    out.push_back(std::move(b));
  }
  std::fclose(f);
  return out;
}

static uint32_t g_encoding = CRR_ENCODING_THRIFTRW;  // argv[3] == "json": every blob json-encoded

static int decode(const std::vector<std::vector<uint8_t>>& blobs, int threads) {
  std::vector<const uint8_t*> p;
  std::vector<uint32_t> enc(blobs.size(), g_encoding);
  std::vector<uint64_t> len;
  std::vector<crr_wf_source> wf;
  for (size_t i = 0; i < blobs.size(); ++i) {
    p.push_back(blobs[i].empty() ? nullptr : blobs[i].data());
    len.push_back(blobs[i].size());
    crr_wf_source s;
    std::memset(&s, 0, sizeof(s));
    s.blob_begin = (uint32_t)i;
    s.blob_count = 1;
    s.run_id = "run";
    s.branch_id = "branch";
    s.new_run_wf = -1;
    wf.push_back(s);
  }
  int err = 0;
  int64_t bad = -1;
  const char* known[] = {"domain-a", "domain-b"};
  crr_decoded* d = crr_decode_histories_enc(p.data(), len.data(), enc.data(), (uint32_t)p.size(), wf.data(),
                                            (uint32_t)wf.size(), known, 2, threads, &err, &bad);
  if (!d) return err;
  crr_decoded_view v;
  crr_decoded_get_view(d, &v);
  volatile uint64_t sink = 0;
  for (uint64_t i = 0; i < v.n_events; ++i) sink += (uint64_t)v.ev.event_id[i] + v.ev.etype[i] + v.key_len[i];
  crr_decoded_free(d);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 2000;
  if (argc > 3 && std::strcmp(argv[3], "json") == 0) g_encoding = CRR_ENCODING_JSON;
  auto corpus = load(argv[1]);
  if (corpus.empty()) { std::fprintf(stderr, "empty corpus\n"); return 2; }
  if (decode(corpus, 4) != 0) { std::fprintf(stderr, "intact corpus failed to decode\n"); return 1; }
  std::mt19937_64 rng(12345);
  int errors = 0, ok = 0;
  for (int r = 0; r < rounds; ++r) {
    std::vector<std::vector<uint8_t>> m;
    for (int k = 0; k < 4; ++k) {
      std::vector<uint8_t> b = corpus[rng() % corpus.size()];
      if (b.empty()) { m.push_back(b); continue; }
      switch (rng() % 4) {
        case 0: b.resize(rng() % b.size()); break;                                  // truncate
        case 1: for (int i = 0; i < 4; ++i) b[rng() % b.size()] ^= (uint8_t)(1u << (rng() % 8)); break;
        case 2: { size_t i = rng() % b.size(); for (int j = 0; j < 4 && i + j < b.size(); ++j) b[i + j] = 0xFF; break; }
        default: b[rng() % b.size()] = (uint8_t)(rng() % 16); break;                // type-byte-like values
      }
      m.push_back(std::move(b));
    }
    (decode(m, 1 + (int)(rng() % 3)) == 0 ? ok : errors)++;
  }
  std::printf("fuzz rounds=%d decoded=%d rejected=%d\n", rounds, ok, errors);
  return 0;
}
