// Native DryadLinqBinary codec + text splitting + Rabin fingerprints (host side).
//
// Byte format: see dryad_amd/io/binary.py (reference LinqToDryad/DryadLinqBinaryWriter.cs,
// DryadLinqBinaryReader.cs).  The native codec works on whole partitions (record streams) and
// converts between the row wire format and column arrays (struct-of-arrays), which is the layout
// the GPU executor uploads to HBM.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dryad {

// Field kinds of a flat record schema.
enum class FieldKind : int {
  U8 = 0, I8 = 1, Bool = 2, I16 = 3, U16 = 4, I32 = 5, U32 = 6, I64 = 7, U64 = 8, F32 = 9, F64 = 10,
  DateTime = 11, Decimal = 12, Guid = 13, String = 14
};

int field_width(FieldKind k);  // bytes, 0 for variable

// Compact int (WriteCompact / ReadCompactInt32).
inline size_t write_compact(uint8_t* p, int32_t v) {
  if (v < 0x80) {
    p[0] = (uint8_t)v;
    return 1;
  }
  p[0] = (uint8_t)(((uint32_t)v >> 24) | 0x80);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
  return 4;
}

// Reads a compact int at p (bounds-checked against end); returns bytes consumed or 0 on EOF.
size_t read_compact(const uint8_t* p, const uint8_t* end, int32_t* v);

// UTF-16 code-unit count of a UTF-8 buffer (surrogate pairs count 2).
int32_t utf16_units(const uint8_t* s, size_t n);

struct StringColumn {
  std::vector<int64_t> offsets;   // n+1 byte offsets into data
  std::vector<uint8_t> data;      // concatenated UTF-8
};

// Decode `n` or all records of a flat schema from a record stream into columns.  Fixed-width
// fields are written into `fixed[i]` (byte buffers, little endian), strings into `strings[i]`.
// Returns the number of records decoded; throws std::runtime_error on a truncated stream.
size_t decode_records(const uint8_t* buf, size_t len, const std::vector<FieldKind>& schema,
                      std::vector<std::vector<uint8_t>>& fixed, std::vector<StringColumn>& strings);

// Encode columns back to a record stream.
std::vector<uint8_t> encode_records(size_t n, const std::vector<FieldKind>& schema,
                                    const std::vector<const uint8_t*>& fixed,
                                    const std::vector<const StringColumn*>& strings);

// Block index of a record stream: offsets[j] = byte offset of record j * block (j = 0, 1, ...),
// found by skipping over fields (string bytes are not touched).  Returns the record count;
// throws std::runtime_error on a truncated stream.  The device decoder (codec.hip) parses every
// block in parallel from these offsets.
size_t scan_record_blocks(const uint8_t* buf, size_t len, const std::vector<FieldKind>& schema, size_t block,
                          std::vector<int64_t>& offsets);

// Split text into lines on \n, \r and \r\n (DryadLinqTextReader.ReadLine semantics).
void split_lines(const uint8_t* buf, size_t len, std::vector<int64_t>& starts, std::vector<int64_t>& ends);

// Text -> LineRecord binary stream (one string record per line).
std::vector<uint8_t> lines_to_records(const uint8_t* buf, size_t len);

// Rabin 64-bit fingerprints over GF(2) with the DryadLINQ polynomial.
class Rabin64 {
 public:
  explicit Rabin64(uint64_t poly = 0x911498ae0e66bad6ull);
  uint64_t empty() const { return poly_; }
  uint64_t extend(uint64_t fp, const uint8_t* data, size_t n) const;
  uint64_t extend_u16(uint64_t fp, uint16_t v) const;
  uint64_t extend_u32(uint64_t fp, uint32_t v) const;
  uint64_t extend_u64(uint64_t fp, uint64_t v) const;
  const uint64_t* table(int b) const { return tab_[b]; }

 private:
  uint64_t poly_;
  uint64_t tab_[8][256];
};

}  // namespace dryad
