// yaml_lite.hpp — the YAML subset of the reference's config files
// (config/world.yml, config/camera.yml: block mappings, block sequences, flow
// sequences of numbers, plain/quoted scalars, comments), resolved the way the
// Python host layer's loader does (PyYAML's YAML 1.1 resolvers plus "1e-5" as
// a float, which is what Ruby's Psych reads; src/configurable_object.rb:43-49).
//
// Duplicate keys keep their first position and take the last value, as Psych
// and PyYAML both do (config/world.yml:40-49 repeats several keys).
#pragma once

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace rtxcli {

struct YNode {
  enum Kind { NUL, SCALAR, SEQ, MAP } kind = NUL;
  std::string s;          // scalar text (quotes removed)
  bool quoted = false;
  std::vector<YNode> seq;
  std::vector<std::pair<std::string, YNode>> map;

  const YNode* get(const std::string& k) const {
    if (kind != MAP) return nullptr;
    for (const auto& kv : map)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

// ---------------------------------------------------------------- scalar typing
enum class SType { Null, Bool, Int, Float, Str };

inline bool all_in(const std::string& s, size_t i, const char* set) {
  if (i >= s.size()) return false;
  for (; i < s.size(); i++)
    if (!strchr(set, s[i])) return false;
  return true;
}

inline std::string strip_us(const std::string& s) {
  std::string o;
  for (char c : s)
    if (c != '_') o += c;
  return o;
}

// YAML 1.1 resolution of a scalar node (PyYAML's implicit resolvers plus the
// loader's extra float form [-+]?digits(.digits)?[eE][-+]?digits).
inline SType classify(const YNode& n) {
  if (n.kind == YNode::NUL) return SType::Null;
  if (n.kind != YNode::SCALAR || n.quoted) return SType::Str;
  const std::string& s = n.s;
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return SType::Null;
  static const char* bools[] = {"yes", "Yes", "YES", "no", "No", "NO", "true", "True", "TRUE",
                                "false", "False", "FALSE", "on", "On", "ON", "off", "Off", "OFF"};
  for (const char* b : bools)
    if (s == b) return SType::Bool;
  const size_t i = (s[0] == '-' || s[0] == '+') ? 1 : 0;
  if (s.compare(i, 2, "0b") == 0 && all_in(s, i + 2, "01_")) return SType::Int;
  if (s.compare(i, 2, "0x") == 0 && all_in(s, i + 2, "0123456789abcdefABCDEF_")) return SType::Int;
  if (i < s.size() && s[i] == '0' && all_in(s, i, "01234567_")) return SType::Int;
  if (i < s.size() && s[i] >= '1' && s[i] <= '9' && all_in(s, i, "0123456789_")) return SType::Int;
  const std::string t = s.substr(i);
  if (t == ".inf" || t == ".Inf" || t == ".INF") return SType::Float;
  if (i == 0 && (t == ".nan" || t == ".NaN" || t == ".NAN")) return SType::Float;
  size_t k = 0, nd = 0, nf = 0;
  while (k < t.size() && (isdigit((unsigned char)t[k]) || (t[k] == '_' && nd))) {
    nd++;
    k++;
  }
  bool dot = false;
  if (k < t.size() && t[k] == '.') {
    dot = true;
    k++;
    while (k < t.size() && (isdigit((unsigned char)t[k]) || t[k] == '_')) {
      nf++;
      k++;
    }
  }
  const bool lead = nd > 0 && isdigit((unsigned char)t[0]);
  if (!(lead || (dot && nf > 0))) return SType::Str;
  if (k == t.size()) return dot ? SType::Float : SType::Str;
  if (t[k] != 'e' && t[k] != 'E') return SType::Str;
  size_t e = k + 1;
  const bool sign = e < t.size() && (t[e] == '-' || t[e] == '+');
  if (sign) e++;
  if (!all_in(t, e, "0123456789")) return SType::Str;
  // PyYAML: a '.' and a signed exponent; the loader's extra rule: leading digits.
  return ((dot && sign) || lead) ? SType::Float : SType::Str;
}

inline bool is_num(const YNode* n) {
  if (!n) return false;
  const SType t = classify(*n);
  return t == SType::Int || t == SType::Float;
}

inline double to_double(const YNode& n) {
  const SType t = classify(n);
  const std::string s = strip_us(n.s);
  const size_t i = (s[0] == '-' || s[0] == '+') ? 1 : 0;
  const bool neg = s[0] == '-';
  if (t == SType::Float) {
    const std::string u = s.substr(i);
    if (u == ".inf" || u == ".Inf" || u == ".INF") return neg ? -HUGE_VAL : HUGE_VAL;
    if (u == ".nan" || u == ".NaN" || u == ".NAN") return NAN;
    return strtod(s.c_str(), nullptr);       // correctly rounded, as Python's float()
  }
  if (t == SType::Int) {
    unsigned long long v;
    if (s.compare(i, 2, "0b") == 0) v = strtoull(s.c_str() + i + 2, nullptr, 2);
    else if (s.compare(i, 2, "0x") == 0) v = strtoull(s.c_str() + i + 2, nullptr, 16);
    else if (s[i] == '0' && s.size() > i + 1) v = strtoull(s.c_str() + i, nullptr, 8);
    else v = strtoull(s.c_str() + i, nullptr, 10);
    return neg ? -(double)v : (double)v;
  }
  throw std::runtime_error("not a number: '" + n.s + "'");
}

// Python truthiness of a loaded value (`x or default`, `if x`).
inline bool truthy(const YNode* n) {
  if (!n) return false;
  switch (classify(*n)) {
    case SType::Null: return false;
    case SType::Bool: {
      const std::string& s = n->s;
      return !(s == "no" || s == "No" || s == "NO" || s == "false" || s == "False" || s == "FALSE" || s == "off" ||
               s == "Off" || s == "OFF");
    }
    case SType::Int:
    case SType::Float: return to_double(*n) != 0.0;
    case SType::Str:
      if (n->kind == YNode::SEQ) return !n->seq.empty();
      if (n->kind == YNode::MAP) return !n->map.empty();
      return !n->s.empty();
  }
  return false;
}

// ---------------------------------------------------------------- parser
class YamlParser {
 public:
  explicit YamlParser(const std::string& text) {
    size_t p = 0;
    int lineno = 0;
    while (p < text.size()) {
      size_t e = text.find('\n', p);
      if (e == std::string::npos) e = text.size();
      std::string ln = text.substr(p, e - p);
      lineno++;
      p = e + 1;
      if (!ln.empty() && ln.back() == '\r') ln.pop_back();
      ln = strip_comment(ln);
      size_t ind = 0;
      while (ind < ln.size() && ln[ind] == ' ') ind++;
      size_t end = ln.size();
      while (end > ind && (ln[end - 1] == ' ' || ln[end - 1] == '\t')) end--;
      if (end == ind) continue;
      if (ln[ind] == '\t') throw err(lineno, "tab indentation");
      const std::string body = ln.substr(ind, end - ind);
      if (body == "---" || body == "...") continue;
      lines_.push_back({(int)ind, body, lineno});
    }
  }

  YNode parse() {
    if (lines_.empty()) return YNode{};
    YNode n = block(lines_[0].indent);
    if (pos_ < lines_.size()) throw err(lines_[pos_].lineno, "unexpected indentation");
    return n;
  }

 private:
  struct Line {
    int indent;
    std::string s;
    int lineno;
  };
  std::vector<Line> lines_;
  size_t pos_ = 0;

  static std::runtime_error err(int lineno, const std::string& m) {
    return std::runtime_error("YAML line " + std::to_string(lineno) + ": " + m);
  }

  static std::string strip_comment(const std::string& ln) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < ln.size(); i++) {
      const char c = ln[i];
      if (c == '\'' && !dq) sq = !sq;
      else if (c == '"' && !sq) dq = !dq;
      else if (c == '#' && !sq && !dq && (i == 0 || ln[i - 1] == ' ' || ln[i - 1] == '\t')) return ln.substr(0, i);
    }
    return ln;
  }

  static bool is_item(const std::string& s) { return s == "-" || s.compare(0, 2, "- ") == 0; }

  // the key/value separator ": " (or a trailing ':') outside quotes and brackets
  static size_t key_sep(const std::string& s) {
    bool sq = false, dq = false;
    int depth = 0;
    for (size_t i = 0; i < s.size(); i++) {
      const char c = s[i];
      if (c == '\'' && !dq) sq = !sq;
      else if (c == '"' && !sq) dq = !dq;
      else if (sq || dq) continue;
      else if (c == '[' || c == '{') depth++;
      else if (c == ']' || c == '}') depth--;
      else if (depth == 0 && c == ':' && (i + 1 == s.size() || s[i + 1] == ' ')) return i;
    }
    return std::string::npos;
  }

  static YNode scalar(const std::string& s) {
    YNode n;
    n.kind = YNode::SCALAR;
    if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\''))) {
      n.quoted = true;
      const char q = s.front();
      for (size_t i = 1; i + 1 < s.size(); i++) {
        if (q == '\'' && s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') {
          n.s += '\'';
          i++;
        } else if (q == '"' && s[i] == '\\' && i + 2 < s.size()) {
          const char c = s[++i];
          n.s += c == 'n' ? '\n' : c == 't' ? '\t' : c;
        } else {
          n.s += s[i];
        }
      }
    } else {
      n.s = s;
    }
    return n;
  }

  YNode flow(const std::string& s, size_t& i, int lineno) {
    YNode n;                                   // s[i] == '['
    n.kind = YNode::SEQ;
    i++;
    while (true) {
      while (i < s.size() && s[i] == ' ') i++;
      if (i >= s.size()) throw err(lineno, "unterminated flow sequence");
      if (s[i] == ']') {
        i++;
        return n;
      }
      if (s[i] == '[') {
        n.seq.push_back(flow(s, i, lineno));
      } else {
        size_t j = i;
        bool sq = false, dq = false;
        while (j < s.size()) {
          if (s[j] == '\'' && !dq) sq = !sq;
          else if (s[j] == '"' && !sq) dq = !dq;
          else if (!sq && !dq && (s[j] == ',' || s[j] == ']')) break;
          j++;
        }
        std::string t = s.substr(i, j - i);
        while (!t.empty() && t.back() == ' ') t.pop_back();
        n.seq.push_back(t.empty() ? YNode{} : scalar(t));
        i = j;
      }
      while (i < s.size() && s[i] == ' ') i++;
      if (i < s.size() && s[i] == ',') i++;
    }
  }

  YNode inline_value(const std::string& s, int lineno) {
    if (!s.empty() && s[0] == '[') {
      size_t i = 0;
      YNode n = flow(s, i, lineno);
      while (i < s.size() && s[i] == ' ') i++;
      if (i != s.size()) throw err(lineno, "text after a flow sequence");
      return n;
    }
    if (!s.empty() && s[0] == '{') throw err(lineno, "flow mappings are not supported");
    return scalar(s);
  }

  YNode block(int indent) {
    if (pos_ >= lines_.size()) return YNode{};
    return is_item(lines_[pos_].s) ? sequence(indent) : mapping(indent);
  }

  YNode sequence(int indent) {
    YNode n;
    n.kind = YNode::SEQ;
    while (pos_ < lines_.size() && lines_[pos_].indent == indent && is_item(lines_[pos_].s)) {
      Line& l = lines_[pos_];
      if (l.s == "-") {
        pos_++;
        if (pos_ < lines_.size() && lines_[pos_].indent > indent) n.seq.push_back(block(lines_[pos_].indent));
        else n.seq.push_back(YNode{});
        continue;
      }
      size_t k = 1;                              // "- rest": rest starts a node at column indent + k
      while (k < l.s.size() && l.s[k] == ' ') k++;
      const std::string rest = l.s.substr(k);
      if (is_item(rest) || (key_sep(rest) != std::string::npos && rest[0] != '[' && rest[0] != '"' &&
                            rest[0] != '\'')) {
        l.indent = indent + (int)k;
        l.s = rest;
        n.seq.push_back(block(l.indent));
      } else {
        pos_++;
        n.seq.push_back(inline_value(rest, l.lineno));
      }
    }
    return n;
  }

  YNode mapping(int indent) {
    YNode n;
    n.kind = YNode::MAP;
    while (pos_ < lines_.size() && lines_[pos_].indent == indent && !is_item(lines_[pos_].s)) {
      const Line l = lines_[pos_];
      const size_t c = key_sep(l.s);
      if (c == std::string::npos) throw err(l.lineno, "expected 'key: value'");
      std::string key = l.s.substr(0, c);
      while (!key.empty() && key.back() == ' ') key.pop_back();
      key = scalar(key).s;
      std::string val = l.s.substr(c + 1);
      size_t b = 0;
      while (b < val.size() && val[b] == ' ') b++;
      val = val.substr(b);
      pos_++;
      YNode v;
      if (!val.empty()) v = inline_value(val, l.lineno);
      else if (pos_ < lines_.size() && lines_[pos_].indent > indent) v = block(lines_[pos_].indent);
      else if (pos_ < lines_.size() && lines_[pos_].indent == indent && is_item(lines_[pos_].s))
        v = sequence(indent);                   // "key:\n- item" at the key's own column
      bool dup = false;
      for (auto& kv : n.map)
        if (kv.first == key) {
          kv.second = v;                        // last value wins, first position kept
          dup = true;
        }
      if (!dup) n.map.emplace_back(key, v);
    }
    if (pos_ < lines_.size() && lines_[pos_].indent > indent)
      throw err(lines_[pos_].lineno, "unexpected indentation");
    return n;
  }
};

inline YNode parse_yaml(const std::string& text) { return YamlParser(text).parse(); }

}  // namespace rtxcli
