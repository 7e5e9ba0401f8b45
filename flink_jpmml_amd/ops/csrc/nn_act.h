// NeuralNetwork activation functions shared by the fused MLP kernel (mlp.hip) and the wide-layer
// GEMM (gemm.hip). Codes mirror runtime/nn_plans.py ACT_CODES.
#pragma once
#include <hip/hip_runtime.h>

enum : int { A_IDENTITY = 0, A_LOGISTIC = 1, A_TANH = 2, A_RELU = 3, A_EXP = 4, A_RECIP = 5, A_SQUARE = 6,
             A_GAUSS = 7, A_SINE = 8, A_COSINE = 9, A_ELLIOTT = 10, A_ARCTAN = 11, A_THRESHOLD = 12 };

__device__ __forceinline__ float activate(int a, float z, float thr) {
  switch (a) {
    case A_LOGISTIC: return 1.0f / (1.0f + __expf(-z));
    case A_TANH: return tanhf(z);
    case A_RELU: return fmaxf(z, 0.0f);
    case A_EXP: return __expf(z);
    case A_RECIP: return 1.0f / z;
    case A_SQUARE: return z * z;
    case A_GAUSS: return __expf(-z * z);
    case A_SINE: return __sinf(z);
    case A_COSINE: return __cosf(z);
    case A_ELLIOTT: return z / (1.0f + fabsf(z));
    case A_ARCTAN: return 0.63661977236758134f * atanf(z);
    case A_THRESHOLD: return z > thr ? 1.0f : 0.0f;
    default: return z;
  }
}
