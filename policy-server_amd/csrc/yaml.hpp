// yaml.hpp — policies.yml (YAML) -> JSON for the native host (src/config.rs:419-453).
#pragma once
#include <cstddef>
#include <string>

namespace kw {

// Converts a YAML document to JSON text; false with a message (and line) on unsupported or
// malformed input.
bool yaml_to_json(const char* text, size_t len, std::string* json, std::string* err);

}  // namespace kw
