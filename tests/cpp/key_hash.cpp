// Prints the reference's Hash_BuiltIn (global.cc:494-497) for keys read from
// stdin: std::hash<std::string> of the decimal key string times the
// coefficient, computed by the toolchain's own libstdc++ (as the reference's
// build computes it).  Used by tests/test_server_group.py.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>

int main(int argc, char** argv) {
  const unsigned coef = argc > 1 ? (unsigned)atoi(argv[1]) : 1u;
  unsigned long long key;
  while (std::scanf("%llu", &key) == 1) {
    const std::string s = std::to_string(key);
    std::printf("%llu\n", (unsigned long long)(std::hash<std::string>()(s) * coef));
  }
  return 0;
}
