// Tiny flag parser shared by the bin/ tools: `--name value [value...]`.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "cpd_api.h"

namespace cli {

struct Args {
    std::map<std::string, std::vector<std::string>> kv;

    Args(int argc, char** argv) {
        std::string key;
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            if (a.rfind("--", 0) == 0) {
                key = a.substr(2);
                kv[key];  // present, maybe without values
            } else if (!key.empty()) {
                kv[key].push_back(a);
            } else {
                std::fprintf(stderr, "unexpected argument '%s'\n", a.c_str());
                std::exit(2);
            }
        }
    }
    bool has(const std::string& k) const { return kv.count(k) > 0; }
    std::string str(const std::string& k, const std::string& def = "") const {
        auto it = kv.find(k);
        return (it == kv.end() || it->second.empty()) ? def : it->second[0];
    }
    std::string str_any(std::initializer_list<const char*> ks, const std::string& def = "") const {
        for (const char* k : ks)
            if (has(k)) return str(k, def);
        return def;
    }
    long long num(const std::string& k, long long def) const {
        std::string s = str(k);
        return s.empty() ? def : std::atoll(s.c_str());
    }
    double real(const std::string& k, double def) const {
        std::string s = str(k);
        return s.empty() ? def : std::atof(s.c_str());
    }
    const std::vector<std::string>& list(const std::string& k) const {
        static const std::vector<std::string> empty;
        auto it = kv.find(k);
        return it == kv.end() ? empty : it->second;
    }
};

inline int method_code(const std::string& m) {
    if (m == "mod") return CPD_PART_MOD;
    if (m == "div") return CPD_PART_DIV;
    std::fprintf(stderr, "partmethod must be 'div' or 'mod', got '%s'\n", m.c_str());
    std::exit(2);
}

inline void check(int rc, const char* what) {
    if (rc != CPD_OK) {
        std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, cpd_last_error());
        std::exit(1);
    }
}

}  // namespace cli
