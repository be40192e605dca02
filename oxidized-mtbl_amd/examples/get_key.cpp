// get-key — examples/get-key.rs over the C++ surface: one Reader::get on the device.
//   usage: get_key <file.mtbl> <key>
#include <cstdio>
#include <fstream>
#include <iterator>

#include "mtbl.hpp"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <file.mtbl> <key>\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", argv[1]);
    return 2;
  }
  const mtbl::Bytes data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const mtbl::Reader reader = mtbl::Reader::open(data);
  const std::string key = argv[2];
  try {
    if (auto v = reader.get(key)) {   // examples/get-key.rs:15-20
      std::printf("\"%s\" \"%.*s\"\n", key.c_str(), (int)v->size(), reinterpret_cast<const char*>(v->data()));
    } else {
      std::printf("entry not found\n");
    }
  } catch (const mtbl::Error& e) {   // `?` returns the Err from main
    std::fprintf(stderr, "Error: Mtbl(%s)\n", e.what());
    return 1;
  }
  return 0;
}
