// Config-file layer of `katago selfplay` (cli_selfplay.cpp): KataGo-style `key = value`
// files (the reference's ConfigParser, core/config_parser.cpp, restricted to what this
// path reads) mapped onto Settings.  Host-only and header-only so the sanitizer build
// (tests/san, tests/test_sanitizers.py) checks the same code the CLI runs.
#pragma once
#include <algorithm>
#include <cstdint>
#include <fstream>
#include <map>
#include <stdexcept>
#include <string>

#include "../../include/katacoffee.h"

namespace kccli {

inline std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

inline bool readConfig(const std::string& path, std::map<std::string, std::string>& kv) {
  std::ifstream in(path);
  if(!in)
    return false;
  std::string line;
  while(std::getline(in, line)) {
    size_t h = line.find('#');
    if(h != std::string::npos)
      line = line.substr(0, h);
    size_t eq = line.find('=');
    if(eq == std::string::npos)
      continue;
    std::string k = trim(line.substr(0, eq)), v = trim(line.substr(eq + 1));
    if(!k.empty())
      kv[k] = v;
  }
  return true;
}

struct Settings {
  int x = 5, y = 5, winLen = 4, games = 4096, gpus = 1, maxRowsPerFile = 10000;
  int servers = 1;  // numNNServerThreadsPerModel: self-play engines (own stream, batch, cache) over all GPUs
  float modelPollSeconds = 10.0f;
  int nnCacheLog2 = 21;  // selfplay1.cfg:121 nnCacheSizePowerOfTwo
  // nnPrecision = auto | corrected | accurate | fast | fastLayered (the reference's useFP16,
  // whose default Auto is mapped to the path within 1e-3 of fp32: corrected / accurate)
  int nnPrecision = COFFEE_NN_DEFAULT;
  int64_t maxGamesTotal = -1;
  uint64_t seed = 0;
  coffee_search_params sp;
};

inline void applyConfig(const std::map<std::string, std::string>& kv, Settings& s) {
  // a value that is not a whole number of the key's type is an error naming the key
  // (the reference's ConfigParser::getInt / getFloat throw IOError the same way)
  auto bad = [](const char* k, const std::string& v) {
    return std::invalid_argument(std::string("config key ") + k + ": bad value '" + v + "'");
  };
  auto parseInt = [&](const char* k, const std::string& v) {
    size_t used = 0;
    int r = 0;
    try {
      r = std::stoi(v, &used);
    } catch(const std::exception&) {
      throw bad(k, v);
    }
    if(used != v.size())
      throw bad(k, v);
    return r;
  };
  auto geti = [&](const char* k, int& v) {
    auto it = kv.find(k);
    if(it != kv.end())
      v = parseInt(k, it->second);
  };
  auto getf = [&](const char* k, float& v) {
    auto it = kv.find(k);
    if(it == kv.end())
      return;
    size_t used = 0;
    try {
      v = std::stof(it->second, &used);
    } catch(const std::exception&) {
      throw bad(k, it->second);
    }
    if(used != it->second.size())
      throw bad(k, it->second);
  };
  auto getb = [&](const char* k, int32_t& v) {
    auto it = kv.find(k);
    if(it != kv.end())
      v = (it->second == "true" || it->second == "True" || it->second == "1") ? 1 : 0;
  };
  auto it = kv.find("bSizes");
  if(it != kv.end())
    s.x = s.y = parseInt("bSizes", trim(it->second.substr(0, it->second.find(','))));
  geti("boardXLen", s.x);
  geti("boardYLen", s.y);
  geti("winLen", s.winLen);
  geti("numGameThreads", s.games);
  geti("numGamesPerGpu", s.games);
  geti("numGpus", s.gpus);
  geti("numNNServerThreadsPerModel", s.servers);
  geti("maxRowsPerTrainFile", s.maxRowsPerFile);
  getf("modelPollSeconds", s.modelPollSeconds);
  geti("nnCacheSizePowerOfTwo", s.nnCacheLog2);  // setup.cpp:268; <= 0 disables the cache
  s.nnCacheLog2 = std::max(0, s.nnCacheLog2);
  it = kv.find("nnPrecision");
  if(it != kv.end()) {
    if(it->second == "auto")
      s.nnPrecision = COFFEE_NN_DEFAULT;
    else if(it->second == "fast")
      s.nnPrecision = COFFEE_NN_FAST;
    else if(it->second == "accurate")
      s.nnPrecision = COFFEE_NN_ACCURATE;
    else if(it->second == "fastLayered")
      s.nnPrecision = COFFEE_NN_FAST_LAYERED;
    else if(it->second == "corrected")
      s.nnPrecision = COFFEE_NN_CORRECTED;
    else
      throw std::invalid_argument("nnPrecision must be auto, corrected, accurate, fast or fastLayered");
  }
  coffee_search_params& p = s.sp;
  geti("maxVisits", p.max_visits);
  getf("cpuctExploration", p.cpuct_exploration);
  getf("cpuctExplorationLog", p.cpuct_exploration_log);
  getf("cpuctExplorationBase", p.cpuct_exploration_base);
  getf("fpuReductionMax", p.fpu_reduction_max);
  getf("rootFpuReductionMax", p.root_fpu_reduction_max);
  getf("fpuLossProp", p.fpu_loss_prop);
  getf("rootFpuLossProp", p.root_fpu_loss_prop);
  getb("fpuParentWeightByVisitedPolicy", p.fpu_parent_weight_by_visited_policy);
  getf("fpuParentWeightByVisitedPolicyPow", p.fpu_parent_weight_by_visited_policy_pow);
  getf("valueWeightExponent", p.value_weight_exponent);
  getb("rootNoiseEnabled", p.root_noise_enabled);
  getf("rootDirichletNoiseTotalConcentration", p.root_dirichlet_noise_total_concentration);
  getf("rootDirichletNoiseWeight", p.root_dirichlet_noise_weight);
  getf("rootPolicyTemperature", p.root_policy_temperature);
  getf("rootPolicyTemperatureEarly", p.root_policy_temperature_early);
  getf("rootDesiredPerChildVisitsCoeff", p.root_desired_per_child_visits_coeff);
  geti("rootNumSymmetriesToSample", p.root_num_symmetries_to_sample);
  getf("chosenMoveTemperature", p.chosen_move_temperature);
  getf("chosenMoveTemperatureEarly", p.chosen_move_temperature_early);
  getf("chosenMoveTemperatureHalflife", p.chosen_move_temperature_halflife);
  getf("chosenMoveSubtract", p.chosen_move_subtract);
  getf("chosenMovePrune", p.chosen_move_prune);
  getb("useLcbForSelection", p.use_lcb_for_selection);
  getf("lcbStdevs", p.lcb_stdevs);
  getf("minVisitPropForLCB", p.min_visit_prop_for_lcb);
  getf("subtreeValueBiasFactor", p.subtree_value_bias_factor);
  getf("subtreeValueBiasWeightExponent", p.subtree_value_bias_weight_exponent);
  getf("subtreeValueBiasFreeProp", p.subtree_value_bias_free_prop);
  getb("useGraphSearch", p.use_graph_search);
  // PlaySettings (playsettings.cpp:80-99)
  getf("cheapSearchProb", p.cheap_search_prob);
  geti("cheapSearchVisits", p.cheap_search_visits);
  getf("cheapSearchTargetWeight", p.cheap_search_target_weight);
  getb("reduceVisits", p.reduce_visits);
  getf("reduceVisitsThreshold", p.reduce_visits_threshold);
  geti("reduceVisitsThresholdLookback", p.reduce_visits_threshold_lookback);
  geti("reducedVisitsMin", p.reduced_visits_min);
  getf("reducedVisitsWeight", p.reduced_visits_weight);
  getf("policySurpriseDataWeight", p.policy_surprise_data_weight);
  getf("valueSurpriseDataWeight", p.value_surprise_data_weight);
  getb("initGamesWithPolicy", p.init_games_with_policy);
  getf("policyInitAreaProp", p.policy_init_area_prop);
  getf("policyInitAreaTemperature", p.policy_init_area_temperature);
  getf("earlyForkGameProb", p.early_fork_game_prob);
  getf("earlyForkGameExpectedMoveProp", p.early_fork_game_expected_move_prop);
  getf("forkGameProb", p.fork_game_prob);
  geti("forkGameMinChoices", p.fork_game_min_choices);
  geti("earlyForkGameMaxChoices", p.early_fork_game_max_choices);
  geti("forkGameMaxChoices", p.fork_game_max_choices);
  getf("sidePositionProb", p.side_position_prob);
  // PlaySettings fields the reference's loader never reads (playsettings.cpp:14): accepted
  // here so the recording can be switched on from a config
  getb("recordTreePositions", p.record_tree_positions);
  geti("recordTreeThreshold", p.record_tree_threshold);
  getf("recordTreeTargetWeight", p.record_tree_target_weight);
}

}  // namespace kccli
