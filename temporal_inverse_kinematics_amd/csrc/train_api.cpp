// train_api.cpp — C ABI of the AmassDataset training-data generation
// (train_data.hip; mmskeleton/datasets/data_amass.py:87-218).
#include <hip/hip_runtime.h>

#include "../../include/tik.h"
#include "common.h"
#include "train_data.h"

using namespace tik_host;

extern "C" {

int tik_rotate_root_z(float* poses, int F, int ld, double angle, void* stream) {
    if (!poses || F < 0 || ld < 3) return fail(TIK_E_INVALID, "tik_rotate_root_z: bad arguments");
    HIP_TRY(tik::launch_rotate_root_z(poses, F, ld, angle, (hipStream_t)stream));
    return TIK_OK;
}

int tik_train_windows(const float* joints, int n_joints, const float* poses, int pose_ld, const int* item_start,
                      const int* item_len, const int* item_idx, const int* item_uid, int B, int h,
                      const int* coco_map, const float* sigma, int relative, int add_noise, unsigned long long seed,
                      float* windows, float* target, void* stream) {
    if (B < 0 || !coco_map || !sigma) return fail(TIK_E_INVALID, "tik_train_windows: bad arguments");
    if (B == 0) return TIK_OK;
    if (!joints || !poses || !item_start || !item_len || !item_idx || !item_uid || !windows || !target ||
        n_joints <= 0 || pose_ld < 66 || h < 0)
        return fail(TIK_E_INVALID, "tik_train_windows: bad arguments");
    if (2 * h + 1 > tik::TW_MAXW) return fail(TIK_E_INVALID, "tik_train_windows: window %d > %d frames", 2 * h + 1, tik::TW_MAXW);
    tik::TrainWinArgs a{};
    a.joints = joints; a.n_joints = n_joints; a.poses = poses; a.pose_ld = pose_ld;
    a.item_start = item_start; a.item_len = item_len; a.item_idx = item_idx; a.item_uid = item_uid;
    a.h = h;
    for (int j = 0; j < 17; ++j) {
        if (coco_map[j] < 0 || coco_map[j] >= n_joints) return fail(TIK_E_INVALID, "tik_train_windows: keypoint map entry %d out of range", j);
        a.map[j] = coco_map[j];
        a.sigma[j] = sigma[j];
    }
    a.relative = relative ? 1 : 0; a.add_noise = add_noise ? 1 : 0; a.seed = seed;
    a.windows = windows; a.target = target;
    HIP_TRY(tik::launch_train_windows(a, B, (hipStream_t)stream));
    return TIK_OK;
}

}  // extern "C"
