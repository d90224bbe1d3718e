// train_data.h — AmassDataset's training-data generation on the GPU (train_data.hip)
#pragma once
#include <hip/hip_runtime.h>

namespace tik {

constexpr int TW_MAXW = 129;   // window frames (h <= 64)

struct TrainWinArgs {
    const float* joints;     // FK joints of all sequences, frames back to back [rows][n_joints][3]
    int n_joints;
    const float* poses;      // pose rows [rows][pose_ld] (first 66 = the target)
    int pose_ld;
    const int* item_start;   // per item: first row of its sequence
    const int* item_len;     // per item: the sequence's frame count
    const int* item_idx;     // per item: the window centre within its sequence
    const int* item_uid;     // per item: the dataset index (noise stream)
    int h;
    int map[17];             // SMPL-X joint of each COCO-17 keypoint
    float sigma[17];         // coco_kps_sigma (data_amass.py:58-62)
    int relative, add_noise;
    unsigned long long seed;
    float* windows;          // [B][2h+1][17][3]
    float* target;           // [B][66]
};

hipError_t launch_rotate_root_z(float* poses, int F, int ld, double angle, hipStream_t st);
hipError_t launch_train_windows(const TrainWinArgs& a, int B, hipStream_t st);

}  // namespace tik
