// Host run of the GPU inflate's decoder (genomeanonymizer_amd/csrc/ganon_inflate.hip, inflate_wave
// with one lane and no barriers): the same source the kernel runs, checked against zlib on the CPU
// by tests/test_inflate.py. Test infrastructure, not part of the product.
//
//   inflate_host_check comp.bin meta.bin out.bin
// meta.bin: int64 n, then n x (int64 in_off, int64 in_len, int64 out_len). out.bin: the blocks'
// outputs back to back (a failed block's bytes are zero). Prints one status per block (0 = ok).
#include "../genomeanonymizer_amd/csrc/ganon_inflate.hip"

#include <cstdio>
#include <memory>

// (ganon_inflate's device path needs it; this harness only runs the decoder on the host)
GANON_API int ganon_batch_sync(ganon_ctx *) { return GANON_E_STATE; }

static std::vector<uint8_t> slurp(const char *p) {
  std::vector<uint8_t> v;
  FILE *f = std::fopen(p, "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  std::fclose(f);
  return v;
}

int main(int argc, char **argv) {
  if (argc != 4) return 2;
  const std::vector<uint8_t> comp = slurp(argv[1]), meta = slurp(argv[2]);
  if (meta.size() < 8) return 2;
  int64_t n;
  std::memcpy(&n, meta.data(), 8);
  if (meta.size() != 8 + 24 * (size_t)n) return 2;
  std::unique_ptr<InfShared> S(new InfShared());
  FILE *fo = std::fopen(argv[3], "wb");
  if (!fo) return 2;
  for (int64_t i = 0; i < n; ++i) {
    int64_t m[3];
    std::memcpy(m, meta.data() + 8 + 24 * i, 24);
    int st = kInfSize;
    std::vector<uint8_t> o((size_t)std::max<int64_t>(m[2], 0), 0);
    if (m[0] >= 0 && m[1] >= 0 && m[0] + m[1] <= (int64_t)comp.size() && m[2] >= 0 && m[2] <= kWin) {
      const int r = inflate_wave<1>(*S, comp.data() + m[0], (int)m[1], o.data(), (int)m[2], 0);
      st = r < 0 ? -r : (r == m[2] ? kInfOk : kInfSize);
    }
    if (st != kInfOk) std::fill(o.begin(), o.end(), 0);
    std::fwrite(o.data(), 1, o.size(), fo);
    std::printf("%d\n", st);
  }
  std::fclose(fo);
  return 0;
}
