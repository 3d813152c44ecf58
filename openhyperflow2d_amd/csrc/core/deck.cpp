#include "deck.hpp"

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace hf2d {

double Table::eval(double xv) const {
  const int n = size();
  if (n == 0) return 0.0;   // the reference's zero table
  if (n == 1) return y[0];
  int i;
  if (xv <= x[0]) {
    i = 1;
  } else if (xv >= x[n - 1]) {
    i = n - 1;
  } else {
    for (i = 1; i < n; i++)
      if (xv >= x[i - 1] && xv < x[i]) break;
  }
  return y[i] + (y[i - 1] - y[i]) * (xv - x[i]) / (x[i - 1] - x[i]);
}

TableData Table::pack() const {
  TableData t;
  if (size() > MAX_TABLE_PTS)
    throw DeckError("table '" + name + "' has more than " + std::to_string(MAX_TABLE_PTS) + " points");
  t.n = size();
  for (int i = 0; i < t.n; i++) {
    t.x[i] = x[i];
    t.y[i] = y[i];
  }
  return t;
}

namespace {

// strtok(buf, "#;") equivalent: skip leading delimiters, then terminate the
// token at the next delimiter.  The buffer start is unchanged, matching the
// reference where subsequent strstr() calls scan from the buffer start.
void cut_comment(std::string& s) {
  size_t i = 0;
  while (i < s.size() && (s[i] == '#' || s[i] == ';')) i++;
  size_t j = s.find_first_of("#;", i);
  if (j != std::string::npos) s.resize(j);
}

bool int_chars_ok(const std::string& v) {
  for (char c : v)
    if (!std::isdigit((unsigned char)c) && c != ' ' && c != '-' && c != '+') return false;
  return true;
}
bool float_chars_ok(const std::string& v) {
  for (char c : v)
    if (!std::isdigit((unsigned char)c) && c != ' ' && c != '-' && c != '+' && c != '.' && c != 'e' &&
        c != 'E')
      return false;
  return true;
}

}  // namespace

InputDeck InputDeck::from_file(const std::string& path) {
  std::ifstream f(path);
  if (!f.is_open()) throw DeckError("Error open data file \"" + path + "\".");
  std::stringstream ss;
  ss << f.rdbuf();
  return from_string(ss.str(), path);
}

InputDeck InputDeck::from_string(const std::string& text, const std::string& origin) {
  InputDeck d;
  d.origin_ = origin;
  std::istringstream in(text);
  std::string raw;
  bool started = false;
  std::string end_tag;
  while (std::getline(in, raw)) {
    if (raw.size() > 1000) raw.resize(1000);   // getline(buf, 1000)
    if (!raw.empty() && raw.back() == '\r') raw.pop_back();
    std::string line = raw;
    cut_comment(line);
    size_t p = line.find("<start/");
    if (p != std::string::npos) {
      if (started) throw DeckError("<start/...> directive defined twice in " + origin);
      size_t e = line.find('>', p);
      d.name_ = line.substr(p + 7, e == std::string::npos ? std::string::npos : e - (p + 7));
      end_tag = "<end/" + d.name_ + ">";
      started = true;
    }
    p = line.find("<data/");
    if (p != std::string::npos) {
      if (!started) throw DeckError("<start/...> directive not found in " + origin);
      size_t eq = line.find('=', p + 6);
      if (eq == std::string::npos) throw DeckError("Error <data/...> directive: " + raw);
      std::string key = line.substr(p + 6, eq - (p + 6));
      // strtok(after '=', ">"): skip leading '>' then read up to next '>'
      size_t v0 = eq + 1;
      while (v0 < line.size() && line[v0] == '>') v0++;
      if (v0 >= line.size()) throw DeckError("Error <data/...> directive: " + raw);
      size_t v1 = line.find('>', v0);
      std::string val = line.substr(v0, v1 == std::string::npos ? std::string::npos : v1 - v0);
      d.data_.push_back({key, val});
    }
    p = line.find("<table=");
    if (p != std::string::npos) {
      if (!started) throw DeckError("<start/...> directive not found in " + origin);
      size_t sl = line.find('/', p + 7);
      if (sl == std::string::npos) throw DeckError("Error <table=.../...> directive: " + raw);
      Table t;
      t.name = line.substr(p + 7, sl - (p + 7));
      size_t gt = line.find('>', sl + 1);
      int n = std::atoi(line.substr(sl + 1, gt == std::string::npos ? std::string::npos : gt - sl - 1).c_str());
      for (int i = 0; i < n; i++) {
        std::string tl;
        if (!std::getline(in, tl)) break;
        if (tl.size() > 1023) tl.resize(1023);
        if (tl.find("<endtable>") != std::string::npos) break;
        size_t sp = tl.find(' ');
        if (sp == std::string::npos) throw DeckError("Error <table=.../...> directive: " + tl);
        t.x.push_back(std::atof(tl.c_str()));
        t.y.push_back(std::atof(tl.c_str() + sp));
      }
      d.tables_.push_back(t);
    }
    if (started && raw.find(end_tag) != std::string::npos && line.find(end_tag) != std::string::npos)
      return d;
  }
  if (!started) throw DeckError("<start/...> directive not found in " + origin);
  throw DeckError("<end/...> directive not found in " + origin);
}

InputDeck::Entry* InputDeck::find(const std::string& key) {
  for (auto& e : data_)
    if (e.key == key) return &e;
  return nullptr;
}
const InputDeck::Entry* InputDeck::find(const std::string& key) const {
  for (auto& e : data_)
    if (e.key == key) return &e;
  return nullptr;
}

bool InputDeck::has(const std::string& key) const { return find(key) != nullptr; }
bool InputDeck::has_table(const std::string& key) const {
  for (auto& t : tables_)
    if (t.name == key) return true;
  return false;
}

int InputDeck::get_int(const std::string& key) {
  Entry* e = find(key);
  if (!e) throw DeckError("Data object \"" + key + "\" not found in \"" + name_ + "\".");
  if (!int_chars_ok(e->value)) throw DeckError("Data object \"" + key + "\" have not INT type.");
  int v = std::atoi(e->value.c_str());
  char buf[64];
  std::snprintf(buf, sizeof buf, "%i", v);
  e->value = buf;
  return v;
}

double InputDeck::get_float(const std::string& key) {
  Entry* e = find(key);
  if (!e) throw DeckError("Data object \"" + key + "\" not found in \"" + name_ + "\".");
  if (!float_chars_ok(e->value)) throw DeckError("Data object \"" + key + "\" have not FLOAT type.");
  double v = std::atof(e->value.c_str());
  char buf[64];
  std::snprintf(buf, sizeof buf, "%g", v);
  e->value = buf;
  return v;
}

std::string InputDeck::get_string(const std::string& key) const {
  const Entry* e = find(key);
  if (!e) throw DeckError("Data object \"" + key + "\" not found in \"" + name_ + "\".");
  return e->value;
}

const Table& InputDeck::get_table(const std::string& key) const {
  for (auto& t : tables_)
    if (t.name == key) return t;
  throw DeckError("Table object \"" + key + "\" not found in \"" + name_ + "\".");
}

int InputDeck::get_int_or(const std::string& key, int def) {
  Entry* e = find(key);
  if (!e || !int_chars_ok(e->value)) return def;
  return get_int(key);
}
double InputDeck::get_float_or(const std::string& key, double def) {
  Entry* e = find(key);
  if (!e || !float_chars_ok(e->value)) return def;
  return get_float(key);
}
std::string InputDeck::get_string_or(const std::string& key, const std::string& def) const {
  const Entry* e = find(key);
  return e ? e->value : def;
}

void InputDeck::set(const std::string& key, const std::string& value) {
  Entry* e = find(key);
  if (e)
    e->value = value;
  else
    data_.push_back({key, value});
}

void InputDeck::set_table(const Table& t) {
  for (auto& x : tables_)
    if (x.name == t.name) {
      x = t;
      return;
    }
  tables_.push_back(t);
}

std::vector<std::string> InputDeck::keys() const {
  std::vector<std::string> k;
  for (auto& e : data_) k.push_back(e.key);
  return k;
}
std::vector<std::string> InputDeck::table_names() const {
  std::vector<std::string> k;
  for (auto& t : tables_) k.push_back(t.name);
  return k;
}

std::string InputDeck::to_text() const {
  std::ostringstream o;
  o.precision(17);
  o << "<start/" << name_ << ">\n";
  for (auto& e : data_) o << "<data/" << e.key << "=" << e.value << ">\n";
  for (auto& t : tables_) {
    o << "<table=" << t.name << "/" << t.size() << ">\n";
    for (int i = 0; i < t.size(); i++) o << t.x[i] << " " << t.y[i] << "\n";
    o << "<endtable>\n";
  }
  o << "<end/" << name_ << ">\n";
  return o.str();
}

}  // namespace hf2d
