// libconfig-subset parser (the reference used libconfig itself, config.c:4-42).
// Grammar handled: groups `name = { ... };` / `name : { ... };`, settings `key = value;`
// (ints, floats, "strings", true/false), comments '#', '//', '/* */'.  Arrays/lists are not used
// by run.conf and are rejected with an error.
#include "channel/config.hpp"

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "channel/common.hpp"

namespace channel {

namespace {
constexpr char kStrTag = '\x01';
}

struct ConfigParser {
  const std::string& s;
  size_t i = 0;
  int line = 1;
  ConfigTree out;
  explicit ConfigParser(const std::string& src) : s(src) {}

  [[noreturn]] void err(const std::string& m) {
    CH_CHECK(false, "config parse error at line " << line << ": " << m);
    std::abort();
  }
  void skip_ws() {
    while (i < s.size()) {
      char c = s[i];
      if (c == '\n') { ++line; ++i; }
      else if (std::isspace(static_cast<unsigned char>(c))) ++i;
      else if (c == '#') { while (i < s.size() && s[i] != '\n') ++i; }
      else if (c == '/' && i + 1 < s.size() && s[i + 1] == '/') { while (i < s.size() && s[i] != '\n') ++i; }
      else if (c == '/' && i + 1 < s.size() && s[i + 1] == '*') {
        i += 2;
        while (i + 1 < s.size() && !(s[i] == '*' && s[i + 1] == '/')) { if (s[i] == '\n') ++line; ++i; }
        if (i + 1 >= s.size()) err("unterminated comment");
        i += 2;
      } else break;
    }
  }
  std::string ident() {
    skip_ws();
    size_t b = i;
    while (i < s.size() && (std::isalnum(static_cast<unsigned char>(s[i])) || s[i] == '_' || s[i] == '-' || s[i] == '*')) ++i;
    if (b == i) err("expected identifier");
    return s.substr(b, i - b);
  }
  std::string value() {
    skip_ws();
    if (i >= s.size()) err("expected value");
    if (s[i] == '"') {
      std::string v(1, kStrTag);
      ++i;
      while (i < s.size() && s[i] != '"') {
        if (s[i] == '\\' && i + 1 < s.size()) { ++i; }
        v.push_back(s[i++]);
      }
      if (i >= s.size()) err("unterminated string");
      ++i;
      // adjacent string literals concatenate (libconfig rule)
      skip_ws();
      while (i < s.size() && s[i] == '"') { std::string more = value(); v += more.substr(1); skip_ws(); }
      return v;
    }
    if (s[i] == '[' || s[i] == '(') err("arrays/lists are not supported");
    size_t b = i;
    while (i < s.size() && s[i] != ';' && s[i] != ',' && s[i] != '}' && s[i] != '\n' && s[i] != '#') ++i;
    std::string v = s.substr(b, i - b);
    while (!v.empty() && std::isspace(static_cast<unsigned char>(v.back()))) v.pop_back();
    if (v.empty()) err("empty value");
    return v;
  }
  void group(const std::string& prefix) {
    while (true) {
      skip_ws();
      if (i >= s.size()) {
        if (!prefix.empty()) err("unterminated group '" + prefix + "'");
        return;
      }
      if (s[i] == '}') {
        if (prefix.empty()) err("unbalanced '}'");
        ++i;
        return;
      }
      std::string name = ident();
      skip_ws();
      if (i >= s.size() || (s[i] != '=' && s[i] != ':')) err("expected '=' or ':' after '" + name + "'");
      ++i;
      skip_ws();
      std::string full = prefix.empty() ? name : prefix + "." + name;
      if (i < s.size() && s[i] == '{') {
        ++i;
        group(full);
      } else {
        out.kv_[full] = value();
      }
      skip_ws();
      if (i < s.size() && (s[i] == ';' || s[i] == ',')) ++i;
    }
  }
};

ConfigTree ConfigTree::parse_string(const std::string& text) {
  ConfigParser p(text);
  p.group("");
  return p.out;
}

ConfigTree ConfigTree::parse_file(const std::string& path) {
  std::ifstream f(path);
  CH_CHECK(f.good(), "cannot open config file '" << path << "'");
  std::stringstream ss;
  ss << f.rdbuf();
  return parse_string(ss.str());
}

bool ConfigTree::has(const std::string& key) const { return kv_.count(key) != 0; }

std::string ConfigTree::get_string(const std::string& key, const std::string& dflt) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) return dflt;
  const std::string& v = it->second;
  if (!v.empty() && v[0] == kStrTag) return v.substr(1);
  return v;
}

long ConfigTree::get_int(const std::string& key, long dflt) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) return dflt;
  std::string v = get_string(key, "");
  char* end = nullptr;
  long r = std::strtol(v.c_str(), &end, 0);
  if (end && *end == 'L') ++end;
  CH_CHECK(end && *end == '\0', "config key '" << key << "' is not an integer: '" << v << "'");
  return r;
}

double ConfigTree::get_double(const std::string& key, double dflt) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) return dflt;
  std::string v = get_string(key, "");
  char* end = nullptr;
  double r = std::strtod(v.c_str(), &end);
  CH_CHECK(end && *end == '\0', "config key '" << key << "' is not a number: '" << v << "'");
  return r;
}

bool ConfigTree::get_bool(const std::string& key, bool dflt) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) return dflt;
  std::string v = get_string(key, "");
  for (auto& c : v) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  if (v == "true" || v == "1" || v == "yes" || v == "on") return true;
  if (v == "false" || v == "0" || v == "no" || v == "off") return false;
  CH_CHECK(false, "config key '" << key << "' is not a boolean: '" << v << "'");
}

void ConfigTree::set(const std::string& key, const std::string& raw_value) {
  std::string v = raw_value;
  if (v.size() >= 2 && v.front() == '"' && v.back() == '"') v = std::string(1, kStrTag) + v.substr(1, v.size() - 2);
  kv_[key] = v;
}

namespace {
// Keys may be given either under "application." (reference layout) or at top level.
std::string pick(const ConfigTree& t, const std::string& k) {
  if (t.has("application." + k)) return "application." + k;
  return k;
}
}  // namespace

Config Config::from_tree(const ConfigTree& t) {
  Config c;
  c.NX = static_cast<int>(t.get_int(pick(t, "NX"), c.NX));
  c.NY = static_cast<int>(t.get_int(pick(t, "NY"), c.NY));
  c.NZ = static_cast<int>(t.get_int(pick(t, "NZ"), c.NZ));
  c.in_G = t.get_string(pick(t, "input.G"), c.in_G);
  c.in_DDV = t.get_string(pick(t, "input.DDV"), c.in_DDV);
  c.in_UMEAN = t.get_string(pick(t, "input.UMEAN"), c.in_UMEAN);
  c.out_G = t.get_string(pick(t, "output.G"), c.out_G);
  c.out_DDV = t.get_string(pick(t, "output.DDV"), c.out_DDV);
  c.out_UMEAN = t.get_string(pick(t, "output.UMEAN"), c.out_UMEAN);
  c.path = t.get_string(pick(t, "path"), c.path);
  c.Re = t.get_double(pick(t, "Re"), c.Re);
  c.Q = t.get_double(pick(t, "Q"), c.Q);
  c.LX = t.get_double(pick(t, "LX"), c.LX);
  c.LZ = t.get_double(pick(t, "LZ"), c.LZ);
  c.stretch = t.get_double(pick(t, "stretch"), c.stretch);
  c.nsteps = t.get_int(pick(t, "nsteps"), c.nsteps);
  c.t_end = t.get_double(pick(t, "t_end"), c.t_end);
  c.cfl = t.get_double(pick(t, "cfl"), c.cfl);
  c.dt_fixed = t.get_double(pick(t, "dt_fixed"), c.dt_fixed);
  c.dt_max = t.get_double(pick(t, "dt_max"), c.dt_max);
  c.cfl_mode = t.get_string(pick(t, "cfl_mode"), c.cfl_mode);
  c.stats_every = static_cast<int>(t.get_int(pick(t, "stats_every"), c.stats_every));
  c.symmetry_every = static_cast<int>(t.get_int(pick(t, "symmetry_every"), c.symmetry_every));
  c.checkpoint_every = static_cast<int>(t.get_int(pick(t, "checkpoint_every"), c.checkpoint_every));
  c.checkpoint_async = t.get_bool(pick(t, "checkpoint_async"), c.checkpoint_async);
  c.log_every = static_cast<int>(t.get_int(pick(t, "log_every"), c.log_every));
  c.precision = t.get_string(pick(t, "precision"), c.precision);
  c.decomposition = t.get_string(pick(t, "decomposition"), c.decomposition);
  c.pr = static_cast<int>(t.get_int(pick(t, "pr"), c.pr));
  c.pc = static_cast<int>(t.get_int(pick(t, "pc"), c.pc));
  c.seed = static_cast<unsigned long long>(t.get_int(pick(t, "seed"), static_cast<long>(c.seed)));
  c.ic = t.get_string(pick(t, "ic"), c.ic);
  c.ic_amplitude = t.get_double(pick(t, "ic_amplitude"), c.ic_amplitude);
  c.forcing = t.get_string(pick(t, "forcing"), c.forcing);
  c.influence = t.get_string(pick(t, "influence"), c.influence);
  c.explicit_d2 = t.get_string(pick(t, "explicit_d2"), c.explicit_d2);
  c.health_check = t.get_bool(pick(t, "health_check"), c.health_check);
  c.health_every = static_cast<int>(t.get_int(pick(t, "health_every"), c.health_every));
  c.on_nan = t.get_string(pick(t, "on_nan"), c.on_nan);
  c.snapshot_every = static_cast<int>(t.get_int(pick(t, "snapshot_every"), c.snapshot_every));
  c.max_rollbacks = static_cast<int>(t.get_int(pick(t, "max_rollbacks"), c.max_rollbacks));
  c.rollback_cfl_factor = t.get_double(pick(t, "rollback_cfl_factor"), c.rollback_cfl_factor);
  c.spectra_every = static_cast<int>(t.get_int(pick(t, "spectra_every"), c.spectra_every));
  c.spectra_planes = t.get_string(pick(t, "spectra_planes"), c.spectra_planes);
  c.log_json = t.get_string(pick(t, "log_json"), c.log_json);
  // Reference semantics: input files given => start from file.
  if (c.in_G != "-" && c.in_DDV != "-" && !t.has(pick(t, "ic"))) c.ic = "file";
  c.validate();
  return c;
}

Config Config::from_file(const std::string& path, const std::vector<std::string>& overrides) {
  ConfigTree t = ConfigTree::parse_file(path);
  for (const auto& o : overrides) {
    auto eq = o.find('=');
    CH_CHECK(eq != std::string::npos, "override '" << o << "' is not key=value");
    std::string k = o.substr(0, eq);
    if (t.has("application." + k)) k = "application." + k;
    t.set(k, o.substr(eq + 1));
  }
  return from_tree(t);
}

std::vector<int> Config::spectra_plane_list() const {
  std::vector<int> out;
  std::string tok;
  std::istringstream is(spectra_planes);
  while (std::getline(is, tok, ',')) {
    tok.erase(0, tok.find_first_not_of(" \t"));
    tok.erase(tok.find_last_not_of(" \t") + 1);
    if (tok.empty()) continue;
    char* end = nullptr;
    const long v = std::strtol(tok.c_str(), &end, 10);
    CH_CHECK(end && *end == '\0', "spectra_planes: '" << tok << "' is not an integer");
    out.push_back(static_cast<int>(v));
  }
  if (out.empty()) out.push_back(NY / 2);
  return out;
}

// transform lengths with kernels (kernels/fft.hip CH_DISPATCH_N): 2^k in [16, 2048], and m*2^k
// (2^k >= 16, at most 2048 points) for m = 3, 5, 7, 9, 11, 13, 15 (the reference's cuFFT plans take
// any length, fft.c:17-23)
bool fft_length_supported(int n) {
  if (n < 16 || n > 2048) return false;
  for (int m : {1, 3, 5, 7, 9, 11, 13, 15}) {
    if (n % m) continue;
    const int p = n / m;
    if ((p & (p - 1)) == 0 && p >= 16) return true;
  }
  return false;
}
static const char* kFftLengths = "2^k (16..2048) or 3, 5, 7, 9, 11, 13, 15 times 2^k >= 16 (at most 2048)";

void Config::validate() const {
  CH_CHECK(fft_length_supported(NX), "NX=" << NX << " must be " << kFftLengths);
  CH_CHECK(NZ >= 9 && fft_length_supported(2 * NZ - 2),
           "2*NZ-2=" << (2 * NZ - 2) << " (physical z points) must be " << kFftLengths);
  CH_CHECK(NY >= 9 && NY <= 64 * 24, "NY=" << NY << " must be in [9, 1536]");
  CH_CHECK(Re > 0 && Q > 0 && LX > 0 && LZ > 0, "Re, Q, LX, LZ must be positive");
  CH_CHECK(stretch > 0, "stretch must be positive");
  CH_CHECK(cfl > 0, "cfl must be positive");
  CH_CHECK(precision == "fp32" || precision == "fp64", "precision must be fp32|fp64");
  CH_CHECK(decomposition == "slab" || decomposition == "pencil", "decomposition must be slab|pencil");
  CH_CHECK(cfl_mode == "corrected" || cfl_mode == "parity", "cfl_mode must be corrected|parity");
  CH_CHECK(forcing == "implicit" || forcing == "parity", "forcing must be implicit|parity");
  CH_CHECK(influence == "discrete" || influence == "analytic", "influence must be discrete|analytic");
  CH_CHECK(explicit_d2 == "compact" || explicit_d2 == "dd", "explicit_d2 must be compact|dd");
  CH_CHECK(ic == "random" || ic == "laminar" || ic == "file" || ic == "os_mode" || ic == "zero",
           "ic must be random|laminar|file|os_mode|zero");
  CH_CHECK(stats_every >= 0 && symmetry_every >= 0 && checkpoint_every >= 0 && log_every >= 0 &&
               spectra_every >= 0 && snapshot_every >= 0 && health_every >= 1,
           "cadences must be >= 0 (health_every >= 1)");
  CH_CHECK(on_nan == "abort" || on_nan == "rollback", "on_nan must be abort|rollback");
  CH_CHECK(rollback_cfl_factor > 0 && rollback_cfl_factor <= 1, "rollback_cfl_factor must be in (0, 1]");
  CH_CHECK(max_rollbacks >= 0, "max_rollbacks must be >= 0");
  for (int j : spectra_plane_list())
    CH_CHECK(j >= 0 && j < NY, "spectra_planes: y index " << j << " outside [0, NY)");
}

std::string Config::to_string() const {
  std::ostringstream o;
  o.precision(17);
  o << "application:\n{\n";
  o << "  NX = " << NX << ";\n  NY = " << NY << ";\n  NZ = " << NZ << ";\n";
  o << "  input:\n  {\n    G = \"" << in_G << "\";\n    DDV = \"" << in_DDV << "\";\n    UMEAN = \"" << in_UMEAN << "\";\n  };\n";
  o << "  output:\n  {\n    G = \"" << out_G << "\";\n    DDV = \"" << out_DDV << "\";\n    UMEAN = \"" << out_UMEAN << "\";\n  };\n";
  o << "  path = \"" << path << "\";\n";
  o << "  Re = " << Re << ";\n  Q = " << Q << ";\n  LX = " << LX << ";\n  LZ = " << LZ << ";\n";
  o << "  stretch = " << stretch << ";\n  nsteps = " << nsteps << ";\n  t_end = " << t_end << ";\n";
  o << "  cfl = " << cfl << ";\n  dt_fixed = " << dt_fixed << ";\n  dt_max = " << dt_max << ";\n";
  o << "  cfl_mode = \"" << cfl_mode << "\";\n";
  o << "  stats_every = " << stats_every << ";\n  symmetry_every = " << symmetry_every << ";\n";
  o << "  checkpoint_every = " << checkpoint_every << ";\n  checkpoint_async = "
    << (checkpoint_async ? "true" : "false") << ";\n  log_every = " << log_every << ";\n";
  o << "  precision = \"" << precision << "\";\n  decomposition = \"" << decomposition << "\";\n";
  o << "  pr = " << pr << ";\n  pc = " << pc << ";\n  seed = " << seed << ";\n";
  o << "  ic = \"" << ic << "\";\n  ic_amplitude = " << ic_amplitude << ";\n";
  o << "  forcing = \"" << forcing << "\";\n  health_check = " << (health_check ? "true" : "false") << ";\n";
  o << "  influence = \"" << influence << "\";\n  explicit_d2 = \"" << explicit_d2 << "\";\n";
  o << "  health_every = " << health_every << ";\n  on_nan = \"" << on_nan << "\";\n";
  o << "  snapshot_every = " << snapshot_every << ";\n  max_rollbacks = " << max_rollbacks << ";\n";
  o << "  rollback_cfl_factor = " << rollback_cfl_factor << ";\n  spectra_every = " << spectra_every << ";\n";
  o << "  spectra_planes = \"" << spectra_planes << "\";\n  log_json = \"" << log_json << "\";\n";
  o << "};\n";
  return o.str();
}

}  // namespace channel
