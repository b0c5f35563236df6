// Test driver: numba_argsort_focus (fastselect_amd/csrc/fs_internal.h) on
// float32 keys read from argv[1]; elements with interest[j] != 0 (argv[2])
// are the focus.  Writes the resulting permutation (int32) to argv[3].
#include <cstdio>
#include <vector>

#include "../../fastselect_amd/csrc/fs_internal.h"

void fs::set_error(const std::string&) {}

int main(int argc, char** argv) {
  if (argc != 4) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  std::vector<float> key;
  float v;
  while (std::fread(&v, 4, 1, f) == 1) key.push_back(v);
  std::fclose(f);
  std::vector<unsigned char> interest(key.size());
  f = std::fopen(argv[2], "rb");
  if (std::fread(interest.data(), 1, interest.size(), f) != interest.size()) return 3;
  std::fclose(f);
  const int64_t n = (int64_t)key.size();
  std::vector<int32_t> R((size_t)n);
  for (int64_t j = 0; j < n; j++) R[j] = (int32_t)j;
  const int rc = fs::numba_argsort_focus(
      n, R.data(), [&](int32_t j) { return key[j]; },
      [&](int64_t lo, int64_t hi) {
        for (int64_t t = lo; t <= hi; t++)
          if (interest[R[t]]) return true;
        return false;
      });
  f = std::fopen(argv[3], "wb");
  std::fwrite(R.data(), 4, R.size(), f);
  std::fclose(f);
  return rc == 0 ? 0 : 1;
}
