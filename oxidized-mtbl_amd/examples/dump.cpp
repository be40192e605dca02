// dump — examples/dump.rs over the C++ surface (include/mtbl.hpp): every record of an .mtbl
// file, one `"key" "value"` line each.  Blocks are framed, CRC-checked and decoded on the GPU.
//   usage: dump <file.mtbl>
#include <cstdio>
#include <fstream>
#include <iterator>

#include "mtbl.hpp"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <file.mtbl>\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", argv[1]);
    return 2;
  }
  const mtbl::Bytes data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::string out;
  try {
    const mtbl::Reader reader = mtbl::Reader::open(data);   // Reader::new(mmap).unwrap()
    mtbl::ReaderIntoIter iter = reader.into_iter();
    while (auto r = iter.next()) {   // examples/dump.rs:14-20
      out += '"';
      out.append(reinterpret_cast<const char*>(r->key), r->key_len);
      out += "\" \"";
      out.append(reinterpret_cast<const char*>(r->val), r->val_len);
      out += "\"\n";
      if (out.size() > (1u << 20)) {
        std::fwrite(out.data(), 1, out.size(), stdout);
        out.clear();
      }
    }
  } catch (const std::exception& e) {   // the reference's unwrap() / panic: message, non-zero exit
    std::fwrite(out.data(), 1, out.size(), stdout);
    std::fprintf(stderr, "dump: %s\n", e.what());
    return 1;
  }
  std::fwrite(out.data(), 1, out.size(), stdout);
  return 0;
}
