// dk_interner.h — the record-ID interner shared by the host-side units (native ingestion,
// the link database): exact UTF-16 record IDs <-> dense u64 ids.  Not part of the ABI.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

struct dk_interner {
  std::unordered_map<std::u16string, uint64_t> ids;
  std::vector<const std::u16string*> strs;  // id -> its ID string (map nodes are stable)
  uint64_t add(std::u16string&& k) {
    const uint64_t id = (uint64_t)strs.size();
    auto it = ids.emplace(std::move(k), id).first;
    strs.push_back(&it->first);
    return id;
  }
};
