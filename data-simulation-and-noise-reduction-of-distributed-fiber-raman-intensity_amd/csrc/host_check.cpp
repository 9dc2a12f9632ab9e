// Host sanitizer driver (make asan): exercises the host-only part of the C ABI -- parameter names,
// packed sizes, BatchNorm folding + fragment packing (pack.cpp), argument checking and error
// reporting (abi.cpp) -- under AddressSanitizer + UndefinedBehaviorSanitizer.  No GPU call is made.
//
//   host_check <arch> <dtype> <tensors.bin> <blob_out.bin>
//
// tensors.bin: for each name of rdn_param_names(arch), in order: int64 numel, then numel float32
// (written by tests/test_abi.py::test_host_sanitizer_pack).  The packed blob is written to
// blob_out.bin so that the test can compare it byte for byte with the library's own rdn_pack.
// Then the error paths: wrong numel, too-small destination, null pointers, bad arch/dtype.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/raman_mi355x.h"

static int fails = 0;
#define EXPECT(c)                                                     \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "host_check: FAILED %s (line %d)\n", #c, __LINE__); \
      ++fails;                                                        \
    }                                                                 \
  } while (0)

int main(int argc, char** argv) {
  if (argc != 5) {
    std::fprintf(stderr, "usage: host_check <arch> <dtype> <tensors.bin> <blob_out.bin>\n");
    return 2;
  }
  const int arch = std::atoi(argv[1]), dtype = std::atoi(argv[2]);
  size_t need = 0;
  EXPECT(rdn_param_names(arch, nullptr, 0, &need) == RDN_OK && need > 1);
  std::string names(need, '\0');
  EXPECT(rdn_param_names(arch, &names[0], need, &need) == RDN_OK);
  // a truncating buffer reports ESIZE and still NUL-terminates
  char small[8];
  EXPECT(rdn_param_names(arch, small, sizeof small, &need) == RDN_ESIZE && small[7] == '\0');
  size_t n_names = 0;
  for (char c : names) n_names += c == '\n';

  std::FILE* f = std::fopen(argv[3], "rb");
  if (!f) return 2;
  std::vector<std::vector<float>> data;
  std::vector<int64_t> numels;
  int64_t ne = 0;
  while (std::fread(&ne, sizeof ne, 1, f) == 1) {
    std::vector<float> t((size_t)ne);
    if (ne && std::fread(t.data(), sizeof(float), (size_t)ne, f) != (size_t)ne) return 2;
    numels.push_back(ne);
    data.push_back(std::move(t));
  }
  std::fclose(f);
  EXPECT(data.size() == n_names);
  std::vector<const float*> ptrs;
  for (auto& t : data) ptrs.push_back(t.data());

  size_t bytes = 0;
  EXPECT(rdn_packed_size(arch, dtype, &bytes) == RDN_OK && bytes > 0);
  std::vector<unsigned char> blob(bytes);
  const int n = (int)ptrs.size();
  EXPECT(rdn_pack(arch, dtype, ptrs.data(), numels.data(), n, blob.data(), bytes) == RDN_OK);
  // exactly-sized heap buffer: ASan flags any write past `bytes`
  {
    unsigned char* exact = (unsigned char*)std::malloc(bytes);
    EXPECT(rdn_pack(arch, dtype, ptrs.data(), numels.data(), n, exact, bytes) == RDN_OK);
    EXPECT(std::memcmp(exact, blob.data(), bytes) == 0);
    std::free(exact);
  }
  std::FILE* o = std::fopen(argv[4], "wb");
  if (!o) return 2;
  std::fwrite(blob.data(), 1, bytes, o);
  std::fclose(o);
  // error paths (they may leave `blob` partially written): every one reports, none writes or reads
  // out of bounds
  EXPECT(rdn_pack(arch, dtype, ptrs.data(), numels.data(), n, blob.data(), bytes - 1) == RDN_ESIZE);
  EXPECT(std::strlen(rdn_last_error()) > 0);
  std::vector<int64_t> bad = numels;
  bad[n / 2] -= 1;
  EXPECT(rdn_pack(arch, dtype, ptrs.data(), bad.data(), n, blob.data(), bytes) == RDN_ESHAPE);
  EXPECT(rdn_pack(arch, dtype, ptrs.data(), numels.data(), n - 1, blob.data(), bytes) == RDN_ESHAPE);
  EXPECT(rdn_pack(arch, dtype, nullptr, numels.data(), n, blob.data(), bytes) == RDN_EINVAL);
  EXPECT(rdn_pack(99, dtype, ptrs.data(), numels.data(), n, blob.data(), bytes) == RDN_EINVAL);
  EXPECT(rdn_pack(arch, 17, ptrs.data(), numels.data(), n, blob.data(), bytes) == RDN_EINVAL);
  EXPECT(rdn_packed_size(arch, dtype, nullptr) == RDN_EINVAL);
  // forward argument checks happen before any HIP call
  EXPECT(rdn_forward(arch, dtype, nullptr, nullptr, nullptr, 1, 100, nullptr, 0, nullptr) == RDN_EINVAL);
  EXPECT(rdn_forward(arch, dtype, blob.data(), (const float*)blob.data(), (float*)blob.data(), -1, 100, nullptr, 0,
                     nullptr) == RDN_EINVAL);
  EXPECT(rdn_forward(arch, dtype, blob.data(), (const float*)blob.data(), (float*)blob.data(), 1, 0, nullptr, 0,
                     nullptr) == RDN_EINVAL);
  EXPECT(rdn_metrics(nullptr, nullptr, 1, 100, nullptr, nullptr, nullptr) == RDN_EINVAL);
  EXPECT(rdn_generate(0, 0, 1, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == RDN_EINVAL);

  if (fails) return 1;
  std::printf("host_check: arch %d dtype %d: %zu tensors, %zu bytes packed, all checks passed\n", arch, dtype,
              (size_t)n, bytes);
  return 0;
}
