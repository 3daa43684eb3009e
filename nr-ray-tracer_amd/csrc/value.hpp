// Document tree shared by the JSON and TOML readers.
//
// The reference deserialises scene files with serde_json / toml into
// `SceneConfig` (packages/ray-tracer/src/scene_config.rs:383-404).  Both
// formats are read here into one ordered tree so that the SceneConfig
// semantics (scene_config.cpp) are written once.  Tables keep document order
// because `Vec<(id, Config)>` order is significant for `instances` (later
// entries may `Ref` earlier ones, scene_config.rs:444-452).
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace nrt {

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct Value {
    enum Kind { Null, Bool, Int, Float, String, Array, Table };
    Kind kind = Null;
    bool b = false;
    int64_t i = 0;
    double f = 0.0;
    std::string s;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> tab;
    // TOML bookkeeping: a table created implicitly by a dotted header may
    // still be defined explicitly later; arrays of tables may be extended.
    bool toml_defined = false;
    bool toml_aot = false;      // array created by [[header]]
    bool toml_inline = false;   // inline table / static array: immutable

    static Value make(Kind k) { Value v; v.kind = k; return v; }

    bool is_null() const { return kind == Null; }
    bool is_number() const { return kind == Int || kind == Float; }
    double number() const {
        if (kind == Float) return f;
        if (kind == Int) return (double)i;
        throw ParseError("expected a number");
    }
    const Value* get(const std::string& key) const {
        if (kind != Table) return nullptr;
        for (auto& kv : tab)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    Value* get_mut(const std::string& key) {
        if (kind != Table) return nullptr;
        for (auto& kv : tab)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    Value& insert(const std::string& key, Value v) {
        tab.emplace_back(key, std::move(v));
        return tab.back().second;
    }
};

Value parse_json(const std::string& text);
Value parse_toml(const std::string& text);

}  // namespace nrt
