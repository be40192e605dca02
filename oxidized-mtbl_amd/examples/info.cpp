// info — examples/info.rs over the C++ surface: Reader::new, then the Metadata footer printed
// as Rust's `{:#?}` prints it (/root/reference/examples/info.rs:12-14, src/metadata.rs:11-24).
//   usage: info <file.mtbl>
#include <cstdio>
#include <fstream>
#include <iterator>

#include "mtbl.hpp"

static const char* compression_name(uint64_t c) {   // src/compression.rs:6-15 (Debug)
  static const char* names[] = {"None", "Snappy", "Zlib", "Lz4", "Lz4hc", "Zstd"};
  return c < 6 ? names[c] : "?";
}

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
  try {
    const mtbl::Reader reader = mtbl::Reader::open(data);   // Reader::new(mmap).unwrap()
    const mtbl::Metadata m = reader.metadata();
    std::printf("Metadata {\n");
    std::printf("    file_version: %s,\n", reader.file_version() == 0 ? "FormatV1" : "FormatV2");
    std::printf("    index_block_offset: %llu,\n", (unsigned long long)m.index_block_offset);
    std::printf("    data_block_size: %llu,\n", (unsigned long long)m.data_block_size);
    std::printf("    compression_algorithm: %s,\n", compression_name(m.compression_algorithm));
    std::printf("    count_entries: %llu,\n", (unsigned long long)m.count_entries);
    std::printf("    count_data_blocks: %llu,\n", (unsigned long long)m.count_data_blocks);
    std::printf("    bytes_data_blocks: %llu,\n", (unsigned long long)m.bytes_data_blocks);
    std::printf("    bytes_index_block: %llu,\n", (unsigned long long)m.bytes_index_block);
    std::printf("    bytes_keys: %llu,\n", (unsigned long long)m.bytes_keys);
    std::printf("    bytes_values: %llu,\n", (unsigned long long)m.bytes_values);
    std::printf("}\n");
  } catch (const mtbl::Error& e) {   // unwrap() on Err panics
    std::fprintf(stderr, "called `Result::unwrap()` on an `Err` value: Mtbl(%s)\n", e.what());
    return 101;
  } catch (const mtbl::Panic& e) {
    std::fprintf(stderr, "panicked: %s\n", e.what());
    return 101;
  }
  return 0;
}
