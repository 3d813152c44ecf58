// InputDeck: parser for the OpenHyperFLOW2D ".dat" input format.
//
// Syntax and coercion rules follow obj_data/obj_data.cpp:570-633 and
// :1124-1435 so that existing decks behave identically:
//  * one <start/NAME> ... <end/NAME> storage block;
//  * <data/KEY=VALUE> scalars stored as strings and coerced on read
//    (int: digits, space, +, - only; float: also '.', 'e', 'E'; atoi/atof
//    semantics, so "-0.1735.3e7" reads as -0.1735);
//  * every numeric read rewrites the stored string with "%i"/"%g" formatting
//    (the reference converts the Data object back to a string), so a second
//    float read of the same key returns the %g-rounded value;
//  * <table=NAME/N> followed by N lines "x y" (y parsed after the first
//    space) and <endtable>;
//  * the line comment cut is strtok(line, "#;") — a ';' or '#' that *starts*
//    a line does not comment it out.
// A missing key raises DeckError (the reference aborts the run).
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "common.hpp"

namespace hf2d {

class DeckError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

struct Table {
  std::string name;
  std::vector<double> x, y;
  int size() const { return (int)x.size(); }
  double eval(double xv) const;   // reference interpolation/extrapolation rule
  double X(int i) const { return (i >= 0 && i < size()) ? x[i] : 0.0; }
  double Y(int i) const { return (i >= 0 && i < size()) ? y[i] : 0.0; }
  TableData pack() const;     // POD copy for device use (<= MAX_TABLE_PTS)
};

class InputDeck {
 public:
  InputDeck() = default;
  static InputDeck from_file(const std::string& path);
  static InputDeck from_string(const std::string& text, const std::string& origin = "<string>");

  const std::string& name() const { return name_; }
  bool has(const std::string& key) const;
  bool has_table(const std::string& key) const;

  int get_int(const std::string& key);
  double get_float(const std::string& key);
  std::string get_string(const std::string& key) const;
  const Table& get_table(const std::string& key) const;

  // Non-throwing variants (return def when the key is absent or malformed).
  int get_int_or(const std::string& key, int def);
  double get_float_or(const std::string& key, double def);
  std::string get_string_or(const std::string& key, const std::string& def) const;

  // Overrides / programmatic construction (used by deck generators).
  void set(const std::string& key, const std::string& value);
  void set_table(const Table& t);

  std::vector<std::string> keys() const;
  std::vector<std::string> table_names() const;
  std::string to_text() const;   // serialise back to .dat syntax

 private:
  struct Entry {
    std::string key;
    std::string value;
  };
  Entry* find(const std::string& key);
  const Entry* find(const std::string& key) const;
  std::string name_;
  std::string origin_;
  std::vector<Entry> data_;
  std::vector<Table> tables_;
};

}  // namespace hf2d
