// Mutation fuzzer for the JPEG host parse (csrc/vf_jpeg_parse.h) -- test infrastructure, built
// by tests/test_jpeg_fuzz.py with g++ -fsanitize=address,undefined (the
// C-ABI host code under sanitizers in CPU tests).  The parse runs on bytes a worker receives
// from the network (inverter.py:31-32; the reference swallows decoder failures at
// worker.py:74-76), so every mutated stream must either be refused or parse into a layout
// whose every byte range lies inside the buffer; ASan / UBSan abort on anything else.
//
//   jpeg_parse_fuzz SEED CASES file.jpg [file.jpg ...]
// prints one JSON line: {"cases": N, "accepted": A, "rejected": R, "tables": T, ...}
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "vf_jpeg_parse.h"

using namespace vf::jpeg;

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0u; }
};

std::vector<uint8_t> read_file(const char *path) {
  std::vector<uint8_t> v;
  FILE *f = std::fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[65536];
  size_t k;
  while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  std::fclose(f);
  return v;
}

// marker segments before SOS: (offset of 0xFF, marker, total length incl. the 2 marker bytes)
struct Seg {
  size_t off;
  int m;
  size_t len;
};
std::vector<Seg> segments(const std::vector<uint8_t> &b) {
  std::vector<Seg> out;
  size_t p = 2;
  while (p + 4 <= b.size() && b[p] == 0xFF) {
    const int m = b[p + 1];
    const size_t len = ((size_t)b[p + 2] << 8) | b[p + 3];
    out.push_back(Seg{p, m, len + 2});
    if (m == 0xDA) break;
    p += len + 2;
  }
  return out;
}

const uint8_t kInteresting[] = {0x00, 0x01, 0x7F, 0x80, 0xFE, 0xFF, 0xC0, 0xC1, 0xC2, 0xC4, 0xD0,
                                0xD7, 0xD8, 0xD9, 0xDA, 0xDB, 0xDD, 0x10, 0x11, 0x22, 0x44, 0x0F};

void mutate(std::vector<uint8_t> &b, const std::vector<std::vector<uint8_t>> &corpus, Rng &r) {
  const int rounds = 1 + (int)r.below(3);
  for (int k = 0; k < rounds && !b.empty(); ++k) {
    const auto segs = segments(b);
    switch (r.below(10)) {
      case 0:  // bit flips anywhere
        for (int i = 0, n = 1 + (int)r.below(8); i < n; ++i) b[r.below((uint32_t)b.size())] ^= (uint8_t)(1u << r.below(8));
        break;
      case 1:  // interesting bytes anywhere
        for (int i = 0, n = 1 + (int)r.below(4); i < n; ++i)
          b[r.below((uint32_t)b.size())] = kInteresting[r.below(sizeof kInteresting)];
        break;
      case 2:  // truncation
        b.resize(r.below((uint32_t)b.size() + 1));
        break;
      case 3: {  // a marker segment's length field
        if (segs.empty()) break;
        const Seg &s = segs[r.below((uint32_t)segs.size())];
        if (s.off + 3 >= b.size()) break;
        const uint32_t v = r.below(4) == 0 ? r.below(65536) : (uint32_t)(s.len - 2 + (int)r.below(9) - 4);
        b[s.off + 2] = (uint8_t)(v >> 8);
        b[s.off + 3] = (uint8_t)v;
        break;
      }
      case 4: {  // bytes inside a header segment (tables, SOF, SOS, DRI fields)
        if (segs.empty()) break;
        const Seg &s = segs[r.below((uint32_t)segs.size())];
        if (s.len <= 4) break;
        for (int i = 0, n = 1 + (int)r.below(6); i < n; ++i) {
          const size_t at = s.off + 4 + r.below((uint32_t)(s.len - 4));
          if (at < b.size()) b[at] = r.below(2) ? (uint8_t)r.next() : kInteresting[r.below(sizeof kInteresting)];
        }
        break;
      }
      case 5: {  // delete or duplicate a whole segment
        if (segs.empty()) break;
        const Seg &s = segs[r.below((uint32_t)segs.size())];
        if (s.off + s.len > b.size()) break;
        std::vector<uint8_t> seg(b.begin() + (long)s.off, b.begin() + (long)(s.off + s.len));
        if (r.below(2)) b.erase(b.begin() + (long)s.off, b.begin() + (long)(s.off + s.len));
        else b.insert(b.begin() + (long)s.off, seg.begin(), seg.end());
        break;
      }
      case 6: {  // splice a chunk of another stream in
        const auto &o = corpus[r.below((uint32_t)corpus.size())];
        if (o.empty()) break;
        const size_t from = r.below((uint32_t)o.size()), n = 1 + r.below((uint32_t)std::min<size_t>(4096, o.size() - from));
        const size_t at = r.below((uint32_t)b.size() + 1);
        b.insert(b.begin() + (long)at, o.begin() + (long)from, o.begin() + (long)(from + n));
        break;
      }
      case 7: {  // SOF dimensions (up to 65535 x 65535) or sampling factors
        for (const Seg &s : segs)
          if ((s.m == 0xC0 || s.m == 0xC1) && s.off + 12 < b.size()) {
            const int which = (int)r.below(3);
            if (which == 0) {
              b[s.off + 5] = (uint8_t)r.next(), b[s.off + 6] = (uint8_t)r.next();
            } else if (which == 1) {
              b[s.off + 7] = (uint8_t)r.next(), b[s.off + 8] = (uint8_t)r.next();
            } else if (s.off + 11 < b.size()) {
              b[s.off + 11] = (uint8_t)r.next();
            }
          }
        break;
      }
      case 8: {  // RSTn markers or stray markers into the entropy-coded data
        size_t sos = 0;
        for (const Seg &s : segs)
          if (s.m == 0xDA) sos = s.off + s.len;
        if (!sos || sos + 2 >= b.size()) break;
        for (int i = 0, n = 1 + (int)r.below(4); i < n; ++i) {
          const size_t at = sos + r.below((uint32_t)(b.size() - sos - 1));
          b[at] = 0xFF;
          b[at + 1] = r.below(3) ? (uint8_t)(0xD0 + r.below(8)) : kInteresting[r.below(sizeof kInteresting)];
        }
        break;
      }
      default: {  // a DRI segment inserted before SOS with a random interval
        size_t sos = 0;
        for (const Seg &s : segs)
          if (s.m == 0xDA) sos = s.off;
        if (!sos) break;
        const uint16_t iv = (uint16_t)r.below(r.below(2) ? 64 : 65536);
        const uint8_t dri[6] = {0xFF, 0xDD, 0x00, 0x04, (uint8_t)(iv >> 8), (uint8_t)iv};
        b.insert(b.begin() + (long)sos, dri, dri + 6);
        break;
      }
    }
  }
}

// Every byte range the decoder's layout would read (prepare_decode in vf_jpeg_host.hip): the
// entropy-coded segments between the restart markers.  Reading them here is what lets ASan see
// a range that leaves the buffer.
uint64_t touch_layout(const uint8_t *b, size_t n, const Parsed &P, const Geom &g) {
  uint64_t sum = 0;
  if (P.scan_off > P.scan_end || P.scan_end > n) std::abort();
  size_t start = P.scan_off;
  for (size_t i = 0; i <= P.rst.size(); ++i) {
    const size_t end = i < P.rst.size() ? P.rst[i].first : P.scan_end;
    if (end > n || start >= end) std::abort();
    for (size_t q = start; q < end; q += 61) sum += b[q];
    sum += b[end - 1];
    if (i < P.rst.size()) {
      if (P.rst[i].second + 2 > n) std::abort();
      start = P.rst[i].second + 2;
    }
  }
  if (g.nblocks <= 0 || g.bpm <= 0 || g.bpm > kMaxBpm) std::abort();
  return sum;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s SEED CASES file.jpg...\n", argv[0]);
    return 2;
  }
  Rng r{std::strtoull(argv[1], nullptr, 0) * 0x9E3779B97F4A7C15ull + 1};
  const long cases = std::strtol(argv[2], nullptr, 0);
  std::vector<std::vector<uint8_t>> corpus;
  for (int i = 3; i < argc; ++i) {
    corpus.push_back(read_file(argv[i]));
    if (corpus.back().empty()) {
      std::fprintf(stderr, "cannot read %s\n", argv[i]);
      return 2;
    }
  }
  long accepted = 0, rejected = 0, header_ok = 0, tables_ok = 0, tables_bad = 0, too_big = 0, originals_ok = 0;
  std::map<std::string, long> reasons;
  uint64_t sink = 0;
  // the unmutated corpus parses (else the fuzzer would only test the first rejection)
  for (const auto &c : corpus) {
    Parsed P;
    Geom g;
    HuffDec dc[3], ac[3];
    HuffSync sdc[3], sac[3];
    uint16_t spair[3][1 << kLook];
    std::string err;
    if (parse_frame(c.data(), c.size(), kDefaultMaxPixels, &P, &g, dc, ac, sdc, sac, spair, &err)) ++originals_ok;
    else std::fprintf(stderr, "corpus file rejected: %s\n", err.c_str());
  }
  // the size limits on a known-good frame: its own pixel count passes, one less is refused,
  // and SOF dimensions past JPEG_MAX_DIMENSION or the default limit are refused
  {
    size_t largest = 0;
    for (size_t i = 1; i < corpus.size(); ++i)
      if (corpus[i].size() > corpus[largest].size()) largest = i;
    std::vector<uint8_t> b = corpus[largest];
    size_t sof = 0;
    for (const Seg &s : segments(b))
      if (s.m == 0xC0 || s.m == 0xC1) sof = s.off;
    if (!sof) return 3;
    auto run = [&](const std::vector<uint8_t> &x, uint64_t limit, std::string *err) {
      Parsed P;
      Geom g;
      HuffDec dc[3], ac[3];
      HuffSync sdc[3], sac[3];
      uint16_t spair[3][1 << kLook];
      return parse_frame(x.data(), x.size(), limit, &P, &g, dc, ac, sdc, sac, spair, err);
    };
    const uint64_t px = (uint64_t)((b[sof + 5] << 8) | b[sof + 6]) * (uint64_t)((b[sof + 7] << 8) | b[sof + 8]);
    std::string e1, e2, e3, e4;
    const bool ok_at = run(b, px, &e1), ok_below = run(b, px - 1, &e2);
    std::vector<uint8_t> big = b;
    big[sof + 5] = big[sof + 6] = big[sof + 7] = big[sof + 8] = 0xFF;  // 65535 x 65535
    const bool ok_big = run(big, ~0ull, &e3);
    big[sof + 5] = big[sof + 7] = 0xFF, big[sof + 6] = big[sof + 8] = 0xDC;  // 65500 x 65500
    const bool ok_max = run(big, kDefaultMaxPixels, &e4);
    std::printf("{\"limit_at\": %d, \"limit_below\": \"%s\", \"dim_65535\": \"%s\", \"dim_65500\": \"%s\"}\n",
                (int)ok_at, e2.c_str(), e3.c_str(), e4.c_str());
    if (!ok_at || ok_below || ok_big || ok_max || e3.find("65500") == std::string::npos ||
        e4.find("limit") == std::string::npos || e2.find("limit") == std::string::npos)
      return 4;
  }
  // seeded edge cases: every corpus frame cut just after an SOS marker whose length field is
  // 2..5 (the segment ends at the buffer's last byte, so a component-count read before the
  // length check reads one byte past the input), each in an exact-size buffer
  long sos_short = 0;
  for (const auto &c : corpus) {
    size_t sos = 0;
    for (const Seg &s : segments(c))
      if (s.m == 0xDA) sos = s.off;
    if (!sos) return 5;
    for (int len = 2; len <= 5; ++len) {
      std::vector<uint8_t> b(c.begin(), c.begin() + (long)sos);
      const uint8_t head[4] = {0xFF, 0xDA, 0x00, (uint8_t)len};
      b.insert(b.end(), head, head + 4);
      for (int k = 2; k < len; ++k) b.push_back(0x03);
      uint8_t *buf = static_cast<uint8_t *>(std::malloc(b.size()));
      std::memcpy(buf, b.data(), b.size());
      Parsed H, P;
      Geom g;
      HuffDec dc[3], ac[3];
      HuffSync sdc[3], sac[3];
      uint16_t spair[3][1 << kLook];
      std::string e1, e2;
      const bool bad = parse(buf, b.size(), &H, &e1, false) != 0 &&
                       !parse_frame(buf, b.size(), kDefaultMaxPixels, &P, &g, dc, ac, sdc, sac, spair, &e2);
      std::free(buf);
      if (!bad) return 6;  // a short SOS must be refused
      ++sos_short;
    }
  }
  std::printf("{\"sos_short_refused\": %ld}\n", sos_short);
  for (long i = 0; i < cases; ++i) {
    std::vector<uint8_t> b = corpus[r.below((uint32_t)corpus.size())];
    mutate(b, corpus, r);
    // exactly n bytes on the heap, so any read past the end is an ASan report
    uint8_t *buf = static_cast<uint8_t *>(std::malloc(b.size() ? b.size() : 1));
    if (!b.empty()) std::memcpy(buf, b.data(), b.size());
    Parsed P;
    Geom g;
    HuffDec dc[3], ac[3];
    HuffSync sdc[3], sac[3];
    uint16_t spair[3][1 << kLook];
    std::string err;
    const uint64_t limit = r.below(8) == 0 ? (uint64_t)r.below(1 << 20) + 1 : kDefaultMaxPixels;
    if (parse_frame(buf, b.size(), limit, &P, &g, dc, ac, sdc, sac, spair, &err)) {
      ++accepted;
      if ((uint64_t)P.w * (uint64_t)P.h > limit || P.w > kMaxDimension || P.h > kMaxDimension) std::abort();
      sink += touch_layout(buf, b.size(), P, g);
    } else {
      ++rejected;
      ++reasons[err.substr(0, 40)];
      if (err.find("limit") != std::string::npos || err.find("65500") != std::string::npos) ++too_big;
    }
    Parsed H;  // the header-only path (vf_jpeg_header)
    std::string herr;
    if (parse(buf, b.size(), &H, &herr, false) == 0) {
      ++header_ok;
      sink += (uint64_t)subsamp_of(H) + (uint64_t)H.w;
    }
    std::free(buf);
    // table construction on raw (bits, vals): every code length histogram, DC and AC
    uint8_t bits[17] = {0}, vals[256];
    if (r.below(2)) {  // a standard table's histogram with one count moved by +-1 (near the edge)
      static const uint8_t *const kStd[4] = {kDcLBits, kDcCBits, kAcLBits, kAcCBits};
      std::memcpy(bits, kStd[r.below(4)], 17);
      const int l = 1 + (int)r.below(16);
      bits[l] = (uint8_t)(bits[l] + (r.below(2) ? 1 : -1));
    } else {
      for (int l = 1; l <= 16; ++l) bits[l] = (uint8_t)(r.below(3) ? r.below(1u << std::min(l, 4)) : r.below(256));
    }
    for (auto &v : vals) v = (uint8_t)r.next();
    HuffDec t;
    HuffSync s;
    uint16_t pr[1 << kLook];
    if (build_tables(bits, vals, r.below(2) == 0, &t, &s, pr)) ++tables_ok;
    else ++tables_bad;
  }
  std::printf("{\"cases\": %ld, \"accepted\": %ld, \"rejected\": %ld, \"too_big\": %ld, \"header_ok\": %ld, "
              "\"tables_ok\": %ld, \"tables_bad\": %ld, \"corpus\": %zu, \"corpus_ok\": %ld, \"reasons\": %zu, \"sink\": %llu}\n",
              cases, accepted, rejected, too_big, header_ok, tables_ok, tables_bad, corpus.size(), originals_ok,
              reasons.size(), (unsigned long long)(sink & 0xFFFF));
  return originals_ok == (long)corpus.size() ? 0 : 1;
}
