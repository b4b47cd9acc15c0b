// OpenCV-compatible YAML FileStorage subset (see sa/filestorage.h).
#include "sa/filestorage.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace sa {

static std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(" \t\r\n");
  return s.substr(a, b - a + 1);
}

static int indent_of(const std::string& s) {
  int i = 0;
  while (i < (int)s.size() && s[i] == ' ') ++i;
  return i;
}

static std::vector<std::string> split_items(const std::string& body) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : body) {
    if (c == ',' || c == '\n' || c == '\r') {
      std::string t = trim(cur);
      if (!t.empty()) out.push_back(t);
      cur.clear();
    } else {
      cur += c;
    }
  }
  std::string t = trim(cur);
  if (!t.empty()) out.push_back(t);
  return out;
}

static double parse_real(const std::string& tok) {
  std::string t = trim(tok);
  if (t == ".Inf" || t == "+.Inf") return INFINITY;
  if (t == "-.Inf") return -INFINITY;
  if (t == ".Nan" || t == ".NaN") return NAN;
  return std::strtod(t.c_str(), nullptr);
}

double FsNode::real() const {
  if (kind == kScalar) return parse_real(scalar);
  if (kind == kSeq && !seq.empty()) return parse_real(seq[0]);
  if (kind == kMat && !mat.empty()) return mat.get(0);
  return 0.0;
}

std::vector<double> FsNode::reals() const {
  std::vector<double> v;
  if (kind == kSeq)
    for (auto& s : seq) v.push_back(parse_real(s));
  else if (kind == kMat)
    for (size_t i = 0; i < mat.total(); ++i) v.push_back(mat.get((int)i));
  else if (kind == kScalar)
    v.push_back(real());
  return v;
}

// collect a flow sequence body starting at `rest` (text after the key's colon), possibly
// continuing over following lines until the closing bracket
static std::string collect_flow(const std::vector<std::string>& lines, size_t& i, const std::string& rest) {
  std::string body = rest;
  size_t lb = body.find('[');
  body = body.substr(lb + 1);
  while (body.find(']') == std::string::npos && i + 1 < lines.size()) body += "\n" + lines[++i];
  return body.substr(0, body.find(']'));
}

void FileStorage::parse(const std::string& text) {
  std::vector<std::string> lines;
  {
    std::stringstream ss(text);
    std::string l;
    while (std::getline(ss, l)) {
      size_t h = l.find('#');
      if (h != std::string::npos && l.compare(0, 5, "%YAML") != 0) l = l.substr(0, h);
      lines.push_back(l);
    }
  }
  for (size_t i = 0; i < lines.size(); ++i) {
    const std::string& l = lines[i];
    std::string t = trim(l);
    if (t.empty() || t[0] == '%' || t == "---" || t == "...") continue;
    if (indent_of(l) != 0) continue;  // nested lines are consumed by their parent
    size_t c = t.find(':');
    if (c == std::string::npos) continue;
    std::string key = trim(t.substr(0, c));
    std::string rest = trim(t.substr(c + 1));
    FsNode node;
    if (rest.rfind("!!opencv-matrix", 0) == 0) {
      int rows = 0, cols = 0;
      std::string dt = "d";
      std::string data;
      while (i + 1 < lines.size() && (indent_of(lines[i + 1]) > 0 || trim(lines[i + 1]).empty())) {
        ++i;
        std::string s = trim(lines[i]);
        if (s.empty()) continue;
        size_t cc = s.find(':');
        if (cc == std::string::npos) continue;
        std::string k = trim(s.substr(0, cc)), v = trim(s.substr(cc + 1));
        if (k == "rows") rows = std::atoi(v.c_str());
        else if (k == "cols") cols = std::atoi(v.c_str());
        else if (k == "dt") dt = v;
        else if (k == "data") data = collect_flow(lines, i, v);
      }
      std::vector<std::string> items = split_items(data);
      int cn = 1;
      char base = dt.empty() ? 'd' : dt.back();
      if (dt.size() > 1 && std::isdigit((unsigned char)dt[0])) cn = std::atoi(dt.c_str());
      int depth = SA_64F;
      switch (base) {
        case 'u': depth = SA_8U; break;
        case 'c': depth = SA_8S; break;
        case 'w': depth = SA_16U; break;
        case 's': depth = SA_16S; break;
        case 'i': depth = SA_32S; break;
        case 'f': depth = SA_32F; break;
        default: depth = SA_64F; break;
      }
      node.kind = FsNode::kMat;
      if (rows > 0 && cols > 0) {
        node.mat.create(rows, cols, sa_maketype(depth, cn));
        const size_t n = (size_t)rows * cols * cn;
        for (size_t k = 0; k < n && k < items.size(); ++k) {
          double v = parse_real(items[k]);
          const int r = (int)(k / (cols * cn)), cc2 = (int)(k % (cols * cn));
          switch (depth) {
            case SA_8U: node.mat.ptr<uint8_t>(r)[cc2] = (uint8_t)v; break;
            case SA_8S: node.mat.ptr<int8_t>(r)[cc2] = (int8_t)v; break;
            case SA_16U: node.mat.ptr<uint16_t>(r)[cc2] = (uint16_t)v; break;
            case SA_16S: node.mat.ptr<int16_t>(r)[cc2] = (int16_t)v; break;
            case SA_32S: node.mat.ptr<int32_t>(r)[cc2] = (int32_t)v; break;
            case SA_32F: node.mat.ptr<float>(r)[cc2] = (float)v; break;
            default: node.mat.ptr<double>(r)[cc2] = v; break;
          }
        }
      }
    } else if (!rest.empty() && rest[0] == '[') {
      node.kind = FsNode::kSeq;
      node.seq = split_items(collect_flow(lines, i, rest));
    } else if (!rest.empty()) {
      node.kind = FsNode::kScalar;
      if (rest.size() >= 2 && rest.front() == '"' && rest.back() == '"') rest = rest.substr(1, rest.size() - 2);
      node.scalar = rest;
    } else {
      // block sequence "- item" lines
      node.kind = FsNode::kSeq;
      while (i + 1 < lines.size() && trim(lines[i + 1]).rfind("- ", 0) == 0) {
        ++i;
        node.seq.push_back(trim(trim(lines[i]).substr(2)));
      }
    }
    if (!nodes_.count(key)) order_.push_back(key);
    nodes_[key] = std::move(node);
  }
}

bool FileStorage::open(const std::string& path, int mode) {
  release();
  path_ = path;
  mode_ = mode;
  if (mode == READ) {
    std::ifstream f(path);
    if (!f.good()) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    parse(ss.str());
    opened_ = true;
  } else {
    out_ = "%YAML:1.0\n---\n";
    opened_ = true;
  }
  return opened_;
}

FileStorage FileStorage::from_string(const std::string& text) {
  FileStorage fs;
  fs.parse(text);
  fs.opened_ = true;
  return fs;
}

void FileStorage::release() {
  if (opened_ && mode_ == WRITE && !path_.empty()) {
    std::ofstream f(path_);
    f << out_;
  }
  opened_ = false;
  nodes_.clear();
  order_.clear();
  if (mode_ == WRITE) out_.clear();
  path_.clear();
}

FsNode FileStorage::operator[](const std::string& key) const {
  auto it = nodes_.find(key);
  return it == nodes_.end() ? FsNode() : it->second;
}

std::string fs_format_double(double v) {
  char buf[64];
  if (std::isnan(v)) return ".Nan";
  if (std::isinf(v)) return v > 0 ? ".Inf" : "-.Inf";
  const double r = std::nearbyint(v);
  if (r == v && std::fabs(v) < 2147483647.0) {
    std::snprintf(buf, sizeof(buf), "%d.", (int)r);
  } else {
    std::snprintf(buf, sizeof(buf), "%.16e", v);
  }
  return buf;
}

static std::string fs_format_float(float v) {
  char buf[64];
  if (std::isnan(v)) return ".Nan";
  if (std::isinf(v)) return v > 0 ? ".Inf" : "-.Inf";
  const double r = std::nearbyint((double)v);
  if (r == (double)v && std::fabs(v) < 2147483647.0) std::snprintf(buf, sizeof(buf), "%d.", (int)r);
  else std::snprintf(buf, sizeof(buf), "%.8e", (double)v);
  return buf;
}

// OpenCV flow-collection emitter: items separated by ", ", a new line (indented `indent`)
// whenever the line would pass column 71.
static void emit_flow(std::string& out, const std::string& head, const std::vector<std::string>& items,
                      int indent) {
  std::string line = head + "[";
  bool first = true;
  for (const auto& it : items) {
    if (!first) line += ",";
    const int new_offset = (int)line.size() + (int)it.size();
    if (!first && new_offset > 71 && new_offset - indent > 10) {
      out += line + "\n";
      line = std::string(indent, ' ') + it;
    } else {
      line += " " + it;
    }
    first = false;
  }
  line += " ]";
  out += line + "\n";
}

void FileStorage::write(const std::string& key, const Mat& m) {
  static const char dts[] = {'u', 'c', 'w', 's', 'i', 'f', 'd'};
  out_ += key + ": !!opencv-matrix\n";
  out_ += "   rows: " + std::to_string(m.rows) + "\n";
  out_ += "   cols: " + std::to_string(m.cols) + "\n";
  std::string dt(1, dts[m.depth()]);
  if (m.channels() > 1) dt = std::to_string(m.channels()) + dt;
  out_ += "   dt: " + dt + "\n";
  std::vector<std::string> items;
  for (int r = 0; r < m.rows; ++r)
    for (int c = 0; c < m.cols * m.channels(); ++c) {
      switch (m.depth()) {
        case SA_64F: items.push_back(fs_format_double(m.ptr<double>(r)[c])); break;
        case SA_32F: items.push_back(fs_format_float(m.ptr<float>(r)[c])); break;
        case SA_8U: items.push_back(std::to_string(m.ptr<uint8_t>(r)[c])); break;
        case SA_16S: items.push_back(std::to_string(m.ptr<int16_t>(r)[c])); break;
        case SA_32S: items.push_back(std::to_string(m.ptr<int32_t>(r)[c])); break;
        default: items.push_back(fs_format_double(m.toF64().ptr<double>(r)[c])); break;
      }
    }
  emit_flow(out_, "   data: ", items, 7);
}

void FileStorage::write(const std::string& key, double v) { out_ += key + ": " + fs_format_double(v) + "\n"; }
void FileStorage::write(const std::string& key, int v) { out_ += key + ": " + std::to_string(v) + "\n"; }
void FileStorage::write(const std::string& key, const std::string& s) { out_ += key + ": \"" + s + "\"\n"; }
void FileStorage::write_seq(const std::string& key, const std::vector<int>& v) {
  std::vector<std::string> items;
  for (int x : v) items.push_back(std::to_string(x));
  emit_flow(out_, key + ": ", items, 3);
}

bool read_string_list(const std::string& path, std::vector<std::string>& out) {
  std::ifstream f(path);
  if (!f.good()) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  size_t a = s.find("<imagelist>");
  size_t b = s.find("</imagelist>");
  if (a == std::string::npos || b == std::string::npos) return false;
  std::stringstream body(s.substr(a + 11, b - a - 11));
  std::string tok;
  out.clear();
  while (body >> tok) {
    if (tok.size() >= 2 && tok.front() == '"' && tok.back() == '"') tok = tok.substr(1, tok.size() - 2);
    out.push_back(tok);
  }
  return true;
}

}  // namespace sa
