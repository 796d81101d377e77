// Test client of the proof reader's AVX-512 u8-array parser (stark::json_u8s_v512, host_json.h):
// one case per stdin line, "max<TAB>text" (the text after the array's '['); prints "null" or
// "ok <count> <end offset> <hex bytes>".  Run only where stark_json_simd_width() is 64.
#include <stdint.h>
#include <stdio.h>

#include <iostream>
#include <string>
#include <vector>

namespace stark {
const char* json_u8s_v512(const char* p, const char* e, uint8_t* out, size_t max, size_t* count);
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    const size_t tab = line.find('\t');
    const size_t max = std::stoul(line.substr(0, tab));
    const std::string text = line.substr(tab + 1);
    std::vector<uint8_t> out(max + 64, 0xEE);
    size_t n = 0;
    const char* r = stark::json_u8s_v512(text.data(), text.data() + text.size(), out.data(), max, &n);
    if (!r) {
      printf("null\n");
      continue;
    }
    for (size_t i = n; i < out.size(); ++i)
      if (out[i] != 0xEE) {
        printf("overwrite\n");
        break;
      }
    printf("ok %zu %zu ", n, (size_t)(r - text.data()));
    for (size_t i = 0; i < n; ++i) printf("%02x", out[i]);
    printf("\n");
  }
  return 0;
}
