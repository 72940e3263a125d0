// tests/cpu_emu/svc_check_emu.cpp -- CPU model of the drop-in service's request
// check (TEST CODE, not the product path; run by tests/test_kernel_emu.py).
//
// One request slot's memory (the 32-dword request block and the 1 KiB body
// area, crc32_kernels.h SvcReq / SvcShared) receives a sequence of JSON-RPC
// requests written as the host writes them (rpccrc_api.cpp svc_crc).  For each
// request, every dword that changed is a word a poll may still read STALE
// (pieces of a read arrive in an order the memory system chooses).  The model
// takes the seq word as current (else the request is not pending) and
// enumerates the stale / current choices of every other changed word -- all of
// them when there are at most 14, else 2^13 seeded draws -- and applies the
// service's acceptance rule (crc32_service.hip) to each mixed read:
//   round 6: svc::word_hash sums over the block (and a longer body's masked
//            words) equal to the tag -- crc32_service_math.h;
//   round 5: the XOR of the 32 block dwords equal to len ^ seq ^ svc_mix(len, seq)
//            for inline bodies, no check for longer ones (restated below).
// A mixed read that is accepted while it differs from the current request in a
// word the answer depends on is a FALSE ACCEPT (the service would return the
// CRC of a mix of two requests).  Output: requests, reads tried, false accepts
// of each rule.  Bodies: consecutive requests on a slot step "id" and one
// parameter together, so two dwords change by the same XOR delta whenever the
// two digits share a byte lane, in pairs of one length;
// the pairs alternate between inline (<= 116 B) and body-area (117 B .. 1 KiB)
// requests.
#include "../../rpc_amd/csrc/crc32_service_math.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

using namespace rpccrc;

namespace {

constexpr uint32_t kInline = 116; // crc32_kernels.h kSvcInline (29 words)
constexpr uint32_t kMaxLen = 1024;

struct Slot {
  uint32_t blk[32];         // dword 0 len, 1 seq, 2..30 inline bytes 0..115, 31 tag
  uint32_t body[kMaxLen / 4]; // the body area (words)
};

// round 5's mix (crc32_kernels.h at 0d84651): fmix32 of seq * golden + len
uint32_t r5_mix(uint32_t len, uint32_t seq) {
  uint32_t h = seq * 0x9E3779B1u + len;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

// The host's writes for one request (rpccrc_api.cpp svc_crc); `r5` writes the
// round-5 tag instead.
void host_write(Slot &s, const std::string &b, uint32_t seq, bool r5) {
  const uint32_t len = (uint32_t)b.size();
  uint8_t *inl = reinterpret_cast<uint8_t *>(&s.blk[2]);
  uint32_t tag;
  if (len <= kInline) {
    memcpy(inl + kInline - len, b.data(), len);
    if (r5) {
      tag = r5_mix(len, seq);
      for (int k = 2; k < 31; ++k) tag ^= s.blk[k];
    } else {
      tag = svc::block_sum(len, seq, &s.blk[2]);
    }
  } else {
    const uint32_t seg = svc::seg_of(len);
    memcpy(reinterpret_cast<uint8_t *>(s.body) + 64 * seg - len, b.data(), len);
    if (r5) {
      tag = s.blk[31]; // round 5 wrote no tag for a longer body
    } else {
      tag = svc::block_sum(len, seq, &s.blk[2]) ^
            svc::body_sum(reinterpret_cast<const uint8_t *>(b.data()), len);
    }
  }
  s.blk[31] = tag;
  s.blk[0] = len;
  s.blk[1] = seq;
}

// The service's decision on a read (rb: block as read, bb: body area as read).
bool accepts(const uint32_t *rb, const uint32_t *bb, bool r5) {
  uint32_t len = rb[0];
  const uint32_t seq = rb[1];
  if (len > kMaxLen) len = kMaxLen;
  const bool inl = len <= kInline;
  if (r5) {
    if (!inl) return true;
    uint32_t x = 0;
    for (int k = 0; k < 32; ++k) x ^= rb[k];
    return x == (len ^ seq ^ r5_mix(len, seq));
  }
  uint32_t x = rb[31];
  for (uint32_t k = 0; k < 31; ++k) x ^= svc::word_hash(rb[k], k);
  if (inl) return x == 0;
  const uint32_t seg = svc::seg_of(len), off0 = 64 * seg - len;
  for (uint32_t j = 0; j < 16 * seg; ++j) x ^= svc::word_hash(bb[j] & svc::keep_mask(4 * j, off0), svc::kHashBodyPos + j);
  return x == 0;
}

// Does the answer from this read differ from the current request's?  The words
// the service uses: len, and the inline words or the body words from the
// body's first byte on (bytes before it are masked).
bool differs_in_use(const uint32_t *rb, const uint32_t *bb, const Slot &cur) {
  if (rb[0] != cur.blk[0]) return true;
  const uint32_t len = cur.blk[0];
  if (len <= kInline) {
    for (uint32_t k = 2 + (kInline - len) / 4; k < 31; ++k)
      if (rb[k] != cur.blk[k]) return true;
    return false;
  }
  const uint32_t seg = svc::seg_of(len), off0 = 64 * seg - len;
  for (uint32_t j = off0 / 4; j < 16 * seg; ++j)
    if (bb[j] != cur.body[j]) return true;
  return false;
}

uint64_t splitmix(uint64_t &x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// A JSON-RPC request as client/rpc_codec.c:17 would print it (cJSON,
// unformatted): the id and the first parameter step together; `pad` grows the
// body (a string parameter) so lengths cross the inline bound.
std::string json_body(uint32_t id, uint32_t pad_len, uint32_t shift) {
  std::string s = "{\"jsonrpc\":\"2.0\",\"method\":\"add\",\"params\":[";
  s += std::to_string(id);
  s += ",\"";
  s += std::string(shift, 'x'); // moves the id digit relative to the param digit's byte lane
  s += "\",\"";
  for (uint32_t k = 0; k < pad_len; ++k) s += (char)('a' + (k * 7) % 26);
  s += "\"],\"id\":";
  s += std::to_string(id);
  s += "}";
  return s;
}

} // namespace

// The check sum of a read is linear in the per-word terms: for a given len as
// read, sum(read) = sum(current) ^ XOR over stale words of (term(old) ^
// term(new)).  The enumeration uses that (O(changed words) per read) and checks
// it against accepts() on the first reads of every request.
struct Terms {
  uint32_t base;               // check sum of the current request under this len
  std::vector<uint32_t> delta; // per changed word
  bool inl_r5_skip;            // round 5, longer body: accepted unchecked
};
Terms terms(const Slot &cur, const Slot &old, const std::vector<int> &ch, uint32_t len, bool r5) {
  Terms t;
  uint32_t rb[32];
  memcpy(rb, cur.blk, sizeof(rb));
  rb[0] = len;
  if (len > kMaxLen) len = kMaxLen;
  const bool inl = len <= kInline;
  t.inl_r5_skip = r5 && !inl;
  const uint32_t seq = rb[1];
  const uint32_t seg = svc::seg_of(len), off0 = 64 * seg - len;
  auto term = [&](int w, uint32_t v) -> uint32_t {
    if (w < 32) {
      if (r5) return v;
      return w == 31 ? v : svc::word_hash(v, (uint32_t)w);
    }
    if (r5 || inl) return 0u; // body words are not read
    const uint32_t j = (uint32_t)(w - 32);
    if (j >= 16 * seg) return 0u;
    return svc::word_hash(v & svc::keep_mask(4 * j, off0), svc::kHashBodyPos + j);
  };
  if (r5) {
    uint32_t x = 0;
    for (int k = 0; k < 32; ++k) x ^= rb[k];
    t.base = x ^ (len ^ seq ^ r5_mix(len, seq));
  } else {
    uint32_t x = 0;
    for (int k = 0; k < 32; ++k) x ^= term(k, rb[k]);
    if (!inl)
      for (uint32_t j = 0; j < 16 * seg; ++j) x ^= term(32 + (int)j, cur.body[j]);
    t.base = x;
  }
  for (int w : ch) {
    if (w == 0) {
      t.delta.push_back(0u); // len: handled by the choice of Terms
      continue;
    }
    const uint32_t ov = w < 32 ? old.blk[w] : old.body[w - 32];
    const uint32_t nv = w < 32 ? cur.blk[w] : cur.body[w - 32];
    t.delta.push_back(term(w, ov) ^ term(w, nv));
  }
  return t;
}

int main(int argc, char **argv) {
  const int nreq = argc > 1 ? atoi(argv[1]) : 600;
  const int kAllMax = 14;          // enumerate every subset up to 2^14 reads
  const uint64_t kDraws = 1u << 13; // else seeded draws
  uint64_t trials[2] = {0, 0}, falses[2] = {0, 0}, r5_inline_falses = 0, crosschecked = 0;
  uint64_t rs = 0x5C4EC4ull;
  for (int r5 = 0; r5 < 2; ++r5) {
    Slot s;
    memset(&s, 0, sizeof(s));
    uint32_t seq = 0;
    for (int i = 0; i < nreq; ++i) {
      // pairs of requests of one length (the second steps the id digits: equal
      // XOR deltas in two dwords when they share a byte lane), inline pairs and
      // body-area pairs alternating; the shift moves the digits' byte lanes
      const uint32_t id = 1 + (uint32_t)(i % 9);
      const uint32_t run = (uint32_t)i / 2;
      const uint32_t pad = (run & 1) ? 80 + (run * 37) % 900 : (run * 13) % 40;
      std::string b = json_body(id, pad, (run / 2) % 4);
      if (b.size() > kMaxLen) b.resize(kMaxLen);
      const Slot old = s;
      host_write(s, b, ++seq, r5 != 0);
      // changed words (block dword k as k, body word j as 32 + j); seq (1) stays current
      std::vector<int> ch;
      for (int k = 0; k < 32; ++k)
        if (k != 1 && old.blk[k] != s.blk[k]) ch.push_back(k);
      for (int j = 0; j < (int)(kMaxLen / 4); ++j)
        if (old.body[j] != s.body[j]) ch.push_back(32 + j);
      const int nc = (int)ch.size();
      const bool len_changed = nc > 0 && ch[0] == 0;
      const Terms tc = terms(s, old, ch, s.blk[0], r5 != 0);
      const Terms ts = len_changed ? terms(s, old, ch, old.blk[0], r5 != 0) : tc;
      // used[c]: the current request's answer depends on changed word c
      std::vector<char> used(nc);
      const uint32_t len = s.blk[0];
      for (int c = 0; c < nc; ++c) {
        const int w = ch[c];
        if (w == 0) used[c] = 1;
        else if (len <= kInline) used[c] = w >= 2 + (int)((kInline - len) / 4) && w < 31;
        else {
          const uint32_t seg = svc::seg_of(len), off0 = 64 * seg - len;
          used[c] = w >= 32 && (uint32_t)(w - 32) >= off0 / 4 && (uint32_t)(w - 32) < 16 * seg;
        }
      }
      const bool all = nc <= kAllMax;
      const uint64_t n = all ? (1ull << nc) : kDraws;
      std::vector<uint64_t> m((nc + 63) / 64 + 1);
      uint32_t rb[32], bb[kMaxLen / 4];
      for (uint64_t t = 1; t < n; ++t) { // t = 0: the current request itself
        if (all) m[0] = t;
        else
          for (auto &x : m) x = splitmix(rs);
        auto stale = [&](int c) { return (m[c / 64] >> (c % 64)) & 1u; };
        const Terms &T = (len_changed && stale(0)) ? ts : tc;
        uint32_t x = T.base;
        bool diff = false;
        for (int c = 0; c < nc; ++c)
          if (stale(c)) {
            x ^= T.delta[c];
            diff = diff || used[c];
          }
        const bool acc = T.inl_r5_skip || x == 0u;
        if (t < 64) { // the linear shortcut against the service rule itself
          memcpy(rb, s.blk, sizeof(rb));
          memcpy(bb, s.body, sizeof(bb));
          for (int c = 0; c < nc; ++c)
            if (stale(c)) {
              const int w = ch[c];
              if (w < 32) rb[w] = old.blk[w];
              else bb[w - 32] = old.body[w - 32];
            }
          if (acc != accepts(rb, bb, r5 != 0) || diff != differs_in_use(rb, bb, s)) {
            fprintf(stderr, "model mismatch: request %d read %llu\n", i, (unsigned long long)t);
            return 3;
          }
          ++crosschecked;
        }
        ++trials[r5];
        if (acc && diff) {
          ++falses[r5];
          // round 5 with an inline body as read: the XOR check itself was fooled
          if (r5 && !T.inl_r5_skip) ++r5_inline_falses;
        }
      }
    }
  }
  printf("requests %d\ncrosschecked %llu\nr6_reads %llu\nr6_false_accepts %llu\nr5_reads %llu\nr5_false_accepts %llu\nr5_inline_false_accepts %llu\n",
         nreq, (unsigned long long)crosschecked, (unsigned long long)trials[0], (unsigned long long)falses[0],
         (unsigned long long)trials[1], (unsigned long long)falses[1], (unsigned long long)r5_inline_falses);
  return 0;
}
