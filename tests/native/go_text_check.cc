// Test driver for cilium_amd/csrc/go_text.h (tests/test_go_text.py): reads
// hex-encoded strings, one per line, and writes "<ToLower hex> <field hex>..."
// per line, so the Python test compares Go's string semantics as the C++
// parsers apply them with the oracle's restatement.
#include <cstdio>
#include <iostream>
#include <string>

#include "go_text.h"

static std::string unhex(const std::string& h) {
  std::string s;
  for (size_t i = 0; i + 1 < h.size(); i += 2) s += (char)std::stoi(h.substr(i, 2), nullptr, 16);
  return s;
}

static std::string hex(const std::string& s) {
  static const char* d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : s) {
    o += d[c >> 4];
    o += d[c & 15];
  }
  return o.empty() ? "-" : o;
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    const std::string s = unhex(line);
    std::string out = hex(cg::go::to_lower(s));
    for (const auto& f : cg::go::fields(s)) out += " " + hex(f);
    std::cout << out << "\n";
  }
  return 0;
}
