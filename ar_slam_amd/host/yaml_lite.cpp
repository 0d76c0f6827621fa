// yaml_lite.cpp -- see yaml_lite.hpp.
#include "yaml_lite.hpp"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace arslam {
namespace yaml {

namespace {

struct Line {
  int indent;
  std::string text;   // without indentation, comment and trailing space
  int lineno;
};

std::string strip_comment(const std::string &s) {
  // a '#' starts a comment at line start or after whitespace, outside quotes
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
  }
  return s;
}

std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}

std::string trim(const std::string &s) {
  size_t a = 0;
  while (a < s.size() && (s[a] == ' ' || s[a] == '\t')) ++a;
  return rtrim(s.substr(a));
}

std::string unquote(const std::string &s, int lineno) {
  if (s.size() >= 2 && s.front() == '"' && s.back() == '"') {
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      char c = s[i];
      if (c == '\\' && i + 2 < s.size()) {
        const char n = s[++i];
        switch (n) {
          case 'n': c = '\n'; break;
          case 't': c = '\t'; break;
          case '"': c = '"'; break;
          case '\\': c = '\\'; break;
          case '/': c = '/'; break;
          default: throw ParseError("line " + std::to_string(lineno) + ": unsupported escape");
        }
      }
      out.push_back(c);
    }
    return out;
  }
  if (s.size() >= 2 && s.front() == '\'' && s.back() == '\'') {
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      out.push_back(s[i]);
      if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') ++i;
    }
    return out;
  }
  return s;
}

Node scalar_node(const std::string &raw, int lineno) {
  Node n;
  const std::string t = trim(raw);
  if (t.empty() || t == "~" || t == "null") return n;
  n.kind = Node::Scalar;
  n.scalar = unquote(t, lineno);
  return n;
}

Node flow_seq(const std::string &s, int lineno) {
  // "[a, b, c]" of scalars
  Node n;
  n.kind = Node::Seq;
  std::string body = trim(s.substr(1, s.size() - 2));
  if (body.empty()) return n;
  std::string cur;
  bool sq = false, dq = false;
  for (char c : body) {
    if (c == '\'' && !dq) sq = !sq;
    if (c == '"' && !sq) dq = !dq;
    if (c == ',' && !sq && !dq) {
      n.seq.push_back(scalar_node(cur, lineno));
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  n.seq.push_back(scalar_node(cur, lineno));
  return n;
}

// position of the "key: " separator outside quotes, or npos
size_t key_sep(const std::string &t) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < t.size(); ++i) {
    const char c = t[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (c == ':' && !sq && !dq && (i + 1 == t.size() || t[i + 1] == ' ')) return i;
    else if ((c == '[' || c == '{') && !sq && !dq && i == 0) return std::string::npos;
  }
  return std::string::npos;
}

struct Parser {
  std::vector<Line> lines;
  size_t pos = 0;

  [[noreturn]] void fail(const std::string &msg) {
    const int ln = pos < lines.size() ? lines[pos].lineno : (lines.empty() ? 0 : lines.back().lineno);
    throw ParseError("yaml line " + std::to_string(ln) + ": " + msg);
  }

  Node value_of(const std::string &rest, int indent, int lineno) {
    std::string r = trim(rest);
    if (!r.empty()) {
      if (r.front() == '[') {
        // a flow sequence may continue on more-indented lines (yaml-cpp and
        // PyYAML both wrap long ones): join them until the bracket closes
        while (r.back() != ']' && pos < lines.size() && lines[pos].indent > indent) r += " " + lines[pos++].text;
        if (r.back() != ']') fail("unterminated flow sequence");
        return flow_seq(r, lineno);
      }
      if (r.front() == '{') fail("flow mappings are not supported");
      return scalar_node(r, lineno);
    }
    // nested block (deeper indentation), or a sequence at the same indentation
    if (pos < lines.size() &&
        (lines[pos].indent > indent || (lines[pos].indent == indent && lines[pos].text.rfind("- ", 0) == 0) ||
         (lines[pos].indent == indent && lines[pos].text == "-")))
      return block(lines[pos].indent);
    return Node{};
  }

  Node block(int indent) {
    if (pos >= lines.size()) return Node{};
    const bool is_seq = lines[pos].text == "-" || lines[pos].text.rfind("- ", 0) == 0;
    Node n;
    n.kind = is_seq ? Node::Seq : Node::Map;
    while (pos < lines.size() && lines[pos].indent == indent) {
      Line ln = lines[pos];
      if (is_seq) {
        if (!(ln.text == "-" || ln.text.rfind("- ", 0) == 0)) break;
        std::string item = ln.text == "-" ? "" : trim(ln.text.substr(2));
        ++pos;
        if (item.empty()) {
          n.seq.push_back(value_of("", indent, ln.lineno));
        } else if (key_sep(item) != std::string::npos && item.front() != '"' && item.front() != '\'') {
          // "- key: value" opens a mapping at indent + 2
          const int inner = indent + 2;
          lines.insert(lines.begin() + pos, Line{inner, item, ln.lineno});
          n.seq.push_back(block(inner));
        } else {
          n.seq.push_back(value_of(item, indent, ln.lineno));
        }
      } else {
        const size_t k = key_sep(ln.text);
        if (k == std::string::npos) fail("expected 'key: value'");
        const std::string key = unquote(trim(ln.text.substr(0, k)), ln.lineno);
        ++pos;
        n.map.emplace_back(key, value_of(ln.text.substr(k + 1), indent, ln.lineno));
      }
    }
    if (pos < lines.size() && lines[pos].indent > indent) fail("bad indentation");
    return n;
  }
};

}  // namespace

const Node *Node::find(const std::string &key) const {
  if (kind != Map) return nullptr;
  for (auto &kv : map)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

const Node &Node::operator[](const std::string &key) const {
  const Node *n = find(key);
  if (!n) throw ParseError("missing key '" + key + "'");
  return *n;
}

const Node &Node::operator[](size_t i) const {
  if (kind != Seq || i >= seq.size()) throw ParseError("sequence index out of range");
  return seq[i];
}

double Node::as_double() const {
  if (kind != Scalar) throw ParseError("expected a number");
  const std::string &s = scalar;
  if (s == ".nan" || s == ".NaN" || s == ".NAN") return std::nan("");
  if (s == ".inf" || s == "+.inf" || s == ".Inf") return HUGE_VAL;
  if (s == "-.inf" || s == "-.Inf") return -HUGE_VAL;
  char *end = nullptr;
  errno = 0;
  const double v = std::strtod(s.c_str(), &end);
  if (end == s.c_str() || *end != '\0') throw ParseError("not a number: '" + s + "'");
  return v;
}

long Node::as_long() const {
  if (kind != Scalar) throw ParseError("expected an integer");
  char *end = nullptr;
  const long v = std::strtol(scalar.c_str(), &end, 10);
  if (end == scalar.c_str() || *end != '\0') throw ParseError("not an integer: '" + scalar + "'");
  return v;
}

const std::string &Node::as_string() const {
  if (kind != Scalar) throw ParseError("expected a string");
  return scalar;
}

Node parse(const std::string &text) {
  Parser p;
  std::istringstream in(text);
  std::string raw;
  int lineno = 0;
  while (std::getline(in, raw)) {
    ++lineno;
    if (raw.find('\t') != std::string::npos && raw.find_first_not_of(" \t") != std::string::npos &&
        raw.find_first_not_of(' ') < raw.size() && raw[raw.find_first_not_of(' ')] == '\t')
      throw ParseError("yaml line " + std::to_string(lineno) + ": tab indentation");
    std::string s = rtrim(strip_comment(raw));
    if (trim(s).empty()) continue;
    if (trim(s) == "---" || trim(s) == "...") continue;
    int ind = 0;
    while (ind < (int)s.size() && s[ind] == ' ') ++ind;
    p.lines.push_back(Line{ind, s.substr(ind), lineno});
  }
  if (p.lines.empty()) return Node{};
  Node root = p.block(p.lines[0].indent);
  if (p.pos != p.lines.size()) p.fail("unexpected content");
  return root;
}

Node parse_file(const std::string &path) {
  std::ifstream f(path);
  if (!f) throw ParseError("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return parse(ss.str());
}

std::string format_double(double v) {
  if (std::isnan(v)) return ".nan";
  if (std::isinf(v)) return v > 0 ? ".inf" : "-.inf";
  char buf[40];
  std::snprintf(buf, sizeof(buf), "%.17g", v);
  return buf;
}

std::string quote_if_needed(const std::string &s) {
  bool plain = !s.empty() && s.find_first_of(":#[]{},&*!|>'\"%@`\n") == std::string::npos &&
               s.front() != ' ' && s.back() != ' ' && s.front() != '-' && s != "null" && s != "~";
  if (plain) {
    // a string that would read back as a number keeps its quotes
    char *end = nullptr;
    std::strtod(s.c_str(), &end);
    if (end != s.c_str() && *end == '\0') plain = false;
  }
  if (plain) return s;
  std::string out = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') out.push_back('\\');
    if (c == '\n') { out += "\\n"; continue; }
    out.push_back(c);
  }
  return out + "\"";
}

}  // namespace yaml
}  // namespace arslam
