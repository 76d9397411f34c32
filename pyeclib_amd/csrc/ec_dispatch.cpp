// Field / k dispatch of the region kernels (ec_kernels.hpp, ec_inst.hpp).
#include "ec_kernels.hpp"

#ifdef ECAMD_AB
#include <map>
#include <mutex>
#include <string>
#endif

namespace ecamd {

hipError_t launch_enc16_1(const EncodeParams&, hipStream_t); hipError_t launch_enc16_2(const EncodeParams&, hipStream_t); hipError_t launch_enc16_3(const EncodeParams&, hipStream_t); hipError_t launch_enc16_4(const EncodeParams&, hipStream_t); hipError_t launch_enc16_5(const EncodeParams&, hipStream_t); hipError_t launch_enc16_6(const EncodeParams&, hipStream_t); hipError_t launch_enc16_7(const EncodeParams&, hipStream_t); hipError_t launch_enc16_8(const EncodeParams&, hipStream_t); hipError_t launch_enc16_9(const EncodeParams&, hipStream_t); hipError_t launch_enc16_10(const EncodeParams&, hipStream_t); hipError_t launch_enc16_11(const EncodeParams&, hipStream_t); hipError_t launch_enc16_12(const EncodeParams&, hipStream_t); hipError_t launch_enc16_13(const EncodeParams&, hipStream_t); hipError_t launch_enc16_14(const EncodeParams&, hipStream_t); hipError_t launch_enc16_15(const EncodeParams&, hipStream_t); hipError_t launch_enc16_16(const EncodeParams&, hipStream_t); hipError_t launch_enc16_17(const EncodeParams&, hipStream_t); hipError_t launch_enc16_18(const EncodeParams&, hipStream_t); hipError_t launch_enc16_19(const EncodeParams&, hipStream_t); hipError_t launch_enc16_20(const EncodeParams&, hipStream_t); hipError_t launch_enc16_21(const EncodeParams&, hipStream_t); hipError_t launch_enc16_22(const EncodeParams&, hipStream_t); hipError_t launch_enc16_23(const EncodeParams&, hipStream_t); hipError_t launch_enc16_24(const EncodeParams&, hipStream_t); hipError_t launch_enc16_25(const EncodeParams&, hipStream_t); hipError_t launch_enc16_26(const EncodeParams&, hipStream_t); hipError_t launch_enc16_27(const EncodeParams&, hipStream_t); hipError_t launch_enc16_28(const EncodeParams&, hipStream_t); hipError_t launch_enc16_29(const EncodeParams&, hipStream_t); hipError_t launch_enc16_30(const EncodeParams&, hipStream_t); hipError_t launch_enc16_31(const EncodeParams&, hipStream_t);
hipError_t launch_dec16_1(const DecodeParams&, hipStream_t); hipError_t launch_dec16_2(const DecodeParams&, hipStream_t); hipError_t launch_dec16_3(const DecodeParams&, hipStream_t); hipError_t launch_dec16_4(const DecodeParams&, hipStream_t); hipError_t launch_dec16_5(const DecodeParams&, hipStream_t); hipError_t launch_dec16_6(const DecodeParams&, hipStream_t); hipError_t launch_dec16_7(const DecodeParams&, hipStream_t); hipError_t launch_dec16_8(const DecodeParams&, hipStream_t); hipError_t launch_dec16_9(const DecodeParams&, hipStream_t); hipError_t launch_dec16_10(const DecodeParams&, hipStream_t); hipError_t launch_dec16_11(const DecodeParams&, hipStream_t); hipError_t launch_dec16_12(const DecodeParams&, hipStream_t); hipError_t launch_dec16_13(const DecodeParams&, hipStream_t); hipError_t launch_dec16_14(const DecodeParams&, hipStream_t); hipError_t launch_dec16_15(const DecodeParams&, hipStream_t); hipError_t launch_dec16_16(const DecodeParams&, hipStream_t); hipError_t launch_dec16_17(const DecodeParams&, hipStream_t); hipError_t launch_dec16_18(const DecodeParams&, hipStream_t); hipError_t launch_dec16_19(const DecodeParams&, hipStream_t); hipError_t launch_dec16_20(const DecodeParams&, hipStream_t); hipError_t launch_dec16_21(const DecodeParams&, hipStream_t); hipError_t launch_dec16_22(const DecodeParams&, hipStream_t); hipError_t launch_dec16_23(const DecodeParams&, hipStream_t); hipError_t launch_dec16_24(const DecodeParams&, hipStream_t); hipError_t launch_dec16_25(const DecodeParams&, hipStream_t); hipError_t launch_dec16_26(const DecodeParams&, hipStream_t); hipError_t launch_dec16_27(const DecodeParams&, hipStream_t); hipError_t launch_dec16_28(const DecodeParams&, hipStream_t); hipError_t launch_dec16_29(const DecodeParams&, hipStream_t); hipError_t launch_dec16_30(const DecodeParams&, hipStream_t); hipError_t launch_dec16_31(const DecodeParams&, hipStream_t);
hipError_t launch_enc8_1(const EncodeParams&, hipStream_t); hipError_t launch_enc8_2(const EncodeParams&, hipStream_t); hipError_t launch_enc8_3(const EncodeParams&, hipStream_t); hipError_t launch_enc8_4(const EncodeParams&, hipStream_t); hipError_t launch_enc8_5(const EncodeParams&, hipStream_t); hipError_t launch_enc8_6(const EncodeParams&, hipStream_t); hipError_t launch_enc8_7(const EncodeParams&, hipStream_t); hipError_t launch_enc8_8(const EncodeParams&, hipStream_t); hipError_t launch_enc8_9(const EncodeParams&, hipStream_t); hipError_t launch_enc8_10(const EncodeParams&, hipStream_t); hipError_t launch_enc8_11(const EncodeParams&, hipStream_t); hipError_t launch_enc8_12(const EncodeParams&, hipStream_t); hipError_t launch_enc8_13(const EncodeParams&, hipStream_t); hipError_t launch_enc8_14(const EncodeParams&, hipStream_t); hipError_t launch_enc8_15(const EncodeParams&, hipStream_t); hipError_t launch_enc8_16(const EncodeParams&, hipStream_t); hipError_t launch_enc8_17(const EncodeParams&, hipStream_t); hipError_t launch_enc8_18(const EncodeParams&, hipStream_t); hipError_t launch_enc8_19(const EncodeParams&, hipStream_t); hipError_t launch_enc8_20(const EncodeParams&, hipStream_t); hipError_t launch_enc8_21(const EncodeParams&, hipStream_t); hipError_t launch_enc8_22(const EncodeParams&, hipStream_t); hipError_t launch_enc8_23(const EncodeParams&, hipStream_t); hipError_t launch_enc8_24(const EncodeParams&, hipStream_t); hipError_t launch_enc8_25(const EncodeParams&, hipStream_t); hipError_t launch_enc8_26(const EncodeParams&, hipStream_t); hipError_t launch_enc8_27(const EncodeParams&, hipStream_t); hipError_t launch_enc8_28(const EncodeParams&, hipStream_t); hipError_t launch_enc8_29(const EncodeParams&, hipStream_t); hipError_t launch_enc8_30(const EncodeParams&, hipStream_t); hipError_t launch_enc8_31(const EncodeParams&, hipStream_t);
hipError_t launch_dec8_1(const DecodeParams&, hipStream_t); hipError_t launch_dec8_2(const DecodeParams&, hipStream_t); hipError_t launch_dec8_3(const DecodeParams&, hipStream_t); hipError_t launch_dec8_4(const DecodeParams&, hipStream_t); hipError_t launch_dec8_5(const DecodeParams&, hipStream_t); hipError_t launch_dec8_6(const DecodeParams&, hipStream_t); hipError_t launch_dec8_7(const DecodeParams&, hipStream_t); hipError_t launch_dec8_8(const DecodeParams&, hipStream_t); hipError_t launch_dec8_9(const DecodeParams&, hipStream_t); hipError_t launch_dec8_10(const DecodeParams&, hipStream_t); hipError_t launch_dec8_11(const DecodeParams&, hipStream_t); hipError_t launch_dec8_12(const DecodeParams&, hipStream_t); hipError_t launch_dec8_13(const DecodeParams&, hipStream_t); hipError_t launch_dec8_14(const DecodeParams&, hipStream_t); hipError_t launch_dec8_15(const DecodeParams&, hipStream_t); hipError_t launch_dec8_16(const DecodeParams&, hipStream_t); hipError_t launch_dec8_17(const DecodeParams&, hipStream_t); hipError_t launch_dec8_18(const DecodeParams&, hipStream_t); hipError_t launch_dec8_19(const DecodeParams&, hipStream_t); hipError_t launch_dec8_20(const DecodeParams&, hipStream_t); hipError_t launch_dec8_21(const DecodeParams&, hipStream_t); hipError_t launch_dec8_22(const DecodeParams&, hipStream_t); hipError_t launch_dec8_23(const DecodeParams&, hipStream_t); hipError_t launch_dec8_24(const DecodeParams&, hipStream_t); hipError_t launch_dec8_25(const DecodeParams&, hipStream_t); hipError_t launch_dec8_26(const DecodeParams&, hipStream_t); hipError_t launch_dec8_27(const DecodeParams&, hipStream_t); hipError_t launch_dec8_28(const DecodeParams&, hipStream_t); hipError_t launch_dec8_29(const DecodeParams&, hipStream_t); hipError_t launch_dec8_30(const DecodeParams&, hipStream_t); hipError_t launch_dec8_31(const DecodeParams&, hipStream_t);

static hipError_t dispatch_enc16(const EncodeParams& p, hipStream_t s) {
  switch (p.k) {
    case 1: return launch_enc16_1(p, s);
    case 2: return launch_enc16_2(p, s);
    case 3: return launch_enc16_3(p, s);
    case 4: return launch_enc16_4(p, s);
    case 5: return launch_enc16_5(p, s);
    case 6: return launch_enc16_6(p, s);
    case 7: return launch_enc16_7(p, s);
    case 8: return launch_enc16_8(p, s);
    case 9: return launch_enc16_9(p, s);
    case 10: return launch_enc16_10(p, s);
    case 11: return launch_enc16_11(p, s);
    case 12: return launch_enc16_12(p, s);
    case 13: return launch_enc16_13(p, s);
    case 14: return launch_enc16_14(p, s);
    case 15: return launch_enc16_15(p, s);
    case 16: return launch_enc16_16(p, s);
    case 17: return launch_enc16_17(p, s);
    case 18: return launch_enc16_18(p, s);
    case 19: return launch_enc16_19(p, s);
    case 20: return launch_enc16_20(p, s);
    case 21: return launch_enc16_21(p, s);
    case 22: return launch_enc16_22(p, s);
    case 23: return launch_enc16_23(p, s);
    case 24: return launch_enc16_24(p, s);
    case 25: return launch_enc16_25(p, s);
    case 26: return launch_enc16_26(p, s);
    case 27: return launch_enc16_27(p, s);
    case 28: return launch_enc16_28(p, s);
    case 29: return launch_enc16_29(p, s);
    case 30: return launch_enc16_30(p, s);
    case 31: return launch_enc16_31(p, s);
    default: return hipErrorInvalidValue;
  }
}

static hipError_t dispatch_dec16(const DecodeParams& p, hipStream_t s) {
  switch (p.k) {
    case 1: return launch_dec16_1(p, s);
    case 2: return launch_dec16_2(p, s);
    case 3: return launch_dec16_3(p, s);
    case 4: return launch_dec16_4(p, s);
    case 5: return launch_dec16_5(p, s);
    case 6: return launch_dec16_6(p, s);
    case 7: return launch_dec16_7(p, s);
    case 8: return launch_dec16_8(p, s);
    case 9: return launch_dec16_9(p, s);
    case 10: return launch_dec16_10(p, s);
    case 11: return launch_dec16_11(p, s);
    case 12: return launch_dec16_12(p, s);
    case 13: return launch_dec16_13(p, s);
    case 14: return launch_dec16_14(p, s);
    case 15: return launch_dec16_15(p, s);
    case 16: return launch_dec16_16(p, s);
    case 17: return launch_dec16_17(p, s);
    case 18: return launch_dec16_18(p, s);
    case 19: return launch_dec16_19(p, s);
    case 20: return launch_dec16_20(p, s);
    case 21: return launch_dec16_21(p, s);
    case 22: return launch_dec16_22(p, s);
    case 23: return launch_dec16_23(p, s);
    case 24: return launch_dec16_24(p, s);
    case 25: return launch_dec16_25(p, s);
    case 26: return launch_dec16_26(p, s);
    case 27: return launch_dec16_27(p, s);
    case 28: return launch_dec16_28(p, s);
    case 29: return launch_dec16_29(p, s);
    case 30: return launch_dec16_30(p, s);
    case 31: return launch_dec16_31(p, s);
    default: return hipErrorInvalidValue;
  }
}

static hipError_t dispatch_enc8(const EncodeParams& p, hipStream_t s) {
  switch (p.k) {
    case 1: return launch_enc8_1(p, s);
    case 2: return launch_enc8_2(p, s);
    case 3: return launch_enc8_3(p, s);
    case 4: return launch_enc8_4(p, s);
    case 5: return launch_enc8_5(p, s);
    case 6: return launch_enc8_6(p, s);
    case 7: return launch_enc8_7(p, s);
    case 8: return launch_enc8_8(p, s);
    case 9: return launch_enc8_9(p, s);
    case 10: return launch_enc8_10(p, s);
    case 11: return launch_enc8_11(p, s);
    case 12: return launch_enc8_12(p, s);
    case 13: return launch_enc8_13(p, s);
    case 14: return launch_enc8_14(p, s);
    case 15: return launch_enc8_15(p, s);
    case 16: return launch_enc8_16(p, s);
    case 17: return launch_enc8_17(p, s);
    case 18: return launch_enc8_18(p, s);
    case 19: return launch_enc8_19(p, s);
    case 20: return launch_enc8_20(p, s);
    case 21: return launch_enc8_21(p, s);
    case 22: return launch_enc8_22(p, s);
    case 23: return launch_enc8_23(p, s);
    case 24: return launch_enc8_24(p, s);
    case 25: return launch_enc8_25(p, s);
    case 26: return launch_enc8_26(p, s);
    case 27: return launch_enc8_27(p, s);
    case 28: return launch_enc8_28(p, s);
    case 29: return launch_enc8_29(p, s);
    case 30: return launch_enc8_30(p, s);
    case 31: return launch_enc8_31(p, s);
    default: return hipErrorInvalidValue;
  }
}

static hipError_t dispatch_dec8(const DecodeParams& p, hipStream_t s) {
  switch (p.k) {
    case 1: return launch_dec8_1(p, s);
    case 2: return launch_dec8_2(p, s);
    case 3: return launch_dec8_3(p, s);
    case 4: return launch_dec8_4(p, s);
    case 5: return launch_dec8_5(p, s);
    case 6: return launch_dec8_6(p, s);
    case 7: return launch_dec8_7(p, s);
    case 8: return launch_dec8_8(p, s);
    case 9: return launch_dec8_9(p, s);
    case 10: return launch_dec8_10(p, s);
    case 11: return launch_dec8_11(p, s);
    case 12: return launch_dec8_12(p, s);
    case 13: return launch_dec8_13(p, s);
    case 14: return launch_dec8_14(p, s);
    case 15: return launch_dec8_15(p, s);
    case 16: return launch_dec8_16(p, s);
    case 17: return launch_dec8_17(p, s);
    case 18: return launch_dec8_18(p, s);
    case 19: return launch_dec8_19(p, s);
    case 20: return launch_dec8_20(p, s);
    case 21: return launch_dec8_21(p, s);
    case 22: return launch_dec8_22(p, s);
    case 23: return launch_dec8_23(p, s);
    case 24: return launch_dec8_24(p, s);
    case 25: return launch_dec8_25(p, s);
    case 26: return launch_dec8_26(p, s);
    case 27: return launch_dec8_27(p, s);
    case 28: return launch_dec8_28(p, s);
    case 29: return launch_dec8_29(p, s);
    case 30: return launch_dec8_30(p, s);
    case 31: return launch_dec8_31(p, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream) {
  return p.w == 8 ? dispatch_enc8(p, stream) : dispatch_enc16(p, stream);
}

hipError_t launch_decode(const DecodeParams& p, hipStream_t stream) {
  return p.w == 8 ? dispatch_dec8(p, stream) : dispatch_dec16(p, stream);
}

#ifdef ECAMD_AB
// A/B builds: the launchers' switches, set by name from the A/B tools
// (ecamd_ab_set); unset names read their default.
namespace {
std::mutex g_ab_mu;
std::map<std::string, int> g_ab;
}  // namespace

int ab_knob(const char* name, int dflt) {
  std::lock_guard<std::mutex> lk(g_ab_mu);
  auto it = g_ab.find(name);
  return it == g_ab.end() ? dflt : it->second;
}
#endif

}  // namespace ecamd

#ifdef ECAMD_AB
// Set (value >= 0) or clear (value < 0) an A/B switch; returns 0.
extern "C" int ecamd_ab_set(const char* name, int value) {
  std::lock_guard<std::mutex> lk(ecamd::g_ab_mu);
  if (value < 0)
    ecamd::g_ab.erase(name);
  else
    ecamd::g_ab[name] = value;
  return 0;
}
#endif
