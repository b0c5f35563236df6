#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>
#include <vector>
#include <random>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
#define STREAM(acc, lane16, lane4, laneoff, eb, cb, bp, bstride)  \
  asm volatile(  \
      "s_load_dwordx4 s[40:43], %[cb], 0x0\n"  \
      "s_mov_b64 s[36:37], %[eb]\n"  \
      "s_mov_b64 s[38:39], %[bp]\n"  \
      "s_waitcnt lgkmcnt(0)\n"  \
      "s_mov_b32 s44, s42\n"  \
      "s_mov_b32 s42, s40\n"  \
      "s_mov_b32 s43, s41\n"  \
      "s_mov_b32 s41, s44\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 9f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_waitcnt vmcnt(18)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "7:\n"  \
      "global_load_dwordx2 v[46:47], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(19)\n"  \
      "v_add_u32_dpp v96, v40, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v40, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v40, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v40, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v40, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v40, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v40, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v40, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 64f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "64:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v42, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v42, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v42, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v42, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v42, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v42, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v42, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v42, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 65f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "65:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v42, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v42, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v42, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v42, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v42, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v42, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v42, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v42, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 66f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "66:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v44, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v44, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v44, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v44, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v44, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v44, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v44, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v44, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 67f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "67:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v44, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v44, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v44, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v44, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v44, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v44, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v44, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v44, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v46, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v46, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v46, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v46, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v46, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v46, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v46, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v46, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v46, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v46, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v46, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v46, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v46, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v46, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v46, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v46, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_branch 7b\n"  \
      "8:\n"  \
      "9:\n"  \
      "s_waitcnt vmcnt(0) lgkmcnt(0)\n"  \
      : [acc0] "+v"(acc[0]), [acc1] "+v"(acc[1]), [acc2] "+v"(acc[2]), [acc3] "+v"(acc[3]), [acc4] "+v"(acc[4]), [acc5] "+v"(acc[5]), [acc6] "+v"(acc[6]), [acc7] "+v"(acc[7])  \
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [laneoff] "v"(laneoff), [eb] "s"(eb),  \
        [cb] "s"(cb), [bp] "s"(bp), [bstride] "s"(bstride)  \
      : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127",  \
        "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "scc", "memory")

#define STREAM1(acc, lane16, lane4, laneoff, eb, cb, bp, bstride)  \
  asm volatile(  \
      "s_load_dwordx4 s[40:43], %[cb], 0x0\n"  \
      "s_mov_b64 s[36:37], %[eb]\n"  \
      "s_mov_b64 s[38:39], %[bp]\n"  \
      "s_waitcnt lgkmcnt(0)\n"  \
      "s_mov_b32 s44, s42\n"  \
      "s_mov_b32 s42, s40\n"  \
      "s_mov_b32 s43, s41\n"  \
      "s_mov_b32 s41, s44\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 9f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_waitcnt vmcnt(18)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "7:\n"  \
      "global_load_dwordx2 v[46:47], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(19)\n"  \
      "v_add_u32_dpp v96, v40, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v40, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v40, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v40, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v40, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v40, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v40, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v40, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 64f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "64:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v42, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v42, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v42, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v42, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v42, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v42, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v42, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v42, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 65f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "65:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v42, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v42, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v42, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v42, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v42, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v42, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v42, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v42, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 66f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "66:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v44, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v44, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v44, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v44, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v44, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v44, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v44, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v44, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 67f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "67:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v44, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v44, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v44, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v44, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v44, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v44, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v44, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v44, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v46, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v46, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v46, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v46, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v46, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v46, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v46, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v46, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v46, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v46, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v46, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v46, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v46, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v46, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v46, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v46, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_branch 7b\n"  \
      "8:\n"  \
      "9:\n"  \
      "s_waitcnt vmcnt(0) lgkmcnt(0)\n"  \
      : [acc0] "+v"(acc[0]), [acc1] "+v"(acc[1]), [acc2] "+v"(acc[2]), [acc3] "+v"(acc[3]), [acc4] "+v"(acc[4]), [acc5] "+v"(acc[5]), [acc6] "+v"(acc[6]), [acc7] "+v"(acc[7])  \
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [laneoff] "v"(laneoff), [eb] "s"(eb),  \
        [cb] "s"(cb), [bp] "s"(bp), [bstride] "s"(bstride)  \
      : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127",  \
        "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "scc", "memory")

#define STREAM2(acc, lane16, lane4, laneoff, eb, cb, bp, bstride)  \
  asm volatile(  \
      "s_load_dwordx4 s[40:43], %[cb], 0x0\n"  \
      "s_mov_b64 s[36:37], %[eb]\n"  \
      "s_mov_b64 s[38:39], %[bp]\n"  \
      "s_waitcnt lgkmcnt(0)\n"  \
      "s_mov_b32 s44, s42\n"  \
      "s_mov_b32 s42, s40\n"  \
      "s_mov_b32 s43, s41\n"  \
      "s_mov_b32 s41, s44\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 9f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_waitcnt vmcnt(18)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "7:\n"  \
      "global_load_dwordx2 v[46:47], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32_dpp v96, v40, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v40, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v40, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v40, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v40, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v40, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v40, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v40, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32_dpp v64, v42, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v42, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v42, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v42, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v42, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v42, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v42, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v42, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(9) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32_dpp v96, v42, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v42, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v42, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v42, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v42, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v42, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v42, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v42, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(6) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32_dpp v64, v44, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v44, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v44, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v44, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v44, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v44, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v44, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v44, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(2) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32_dpp v96, v44, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v44, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v44, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v44, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v44, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v44, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v44, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v44, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32_dpp v64, v46, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v46, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v46, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v46, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v46, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v46, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v46, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v46, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32_dpp v96, v46, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v46, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v46, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v46, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v46, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v46, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v46, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v46, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_branch 7b\n"  \
      "8:\n"  \
      "9:\n"  \
      "s_waitcnt vmcnt(0) lgkmcnt(0)\n"  \
      : [acc0] "+v"(acc[0]), [acc1] "+v"(acc[1]), [acc2] "+v"(acc[2]), [acc3] "+v"(acc[3]), [acc4] "+v"(acc[4]), [acc5] "+v"(acc[5]), [acc6] "+v"(acc[6]), [acc7] "+v"(acc[7])  \
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [laneoff] "v"(laneoff), [eb] "s"(eb),  \
        [cb] "s"(cb), [bp] "s"(bp), [bstride] "s"(bstride)  \
      : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127",  \
        "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "scc", "memory")

#define STREAM3(acc, lane16, lane4, laneoff, eb, cb, bp, bstride)  \
  asm volatile(  \
      "s_load_dwordx4 s[40:43], %[cb], 0x0\n"  \
      "s_mov_b64 s[36:37], %[eb]\n"  \
      "s_mov_b64 s[38:39], %[bp]\n"  \
      "s_waitcnt lgkmcnt(0)\n"  \
      "s_mov_b32 s44, s42\n"  \
      "s_mov_b32 s42, s40\n"  \
      "s_mov_b32 s43, s41\n"  \
      "s_mov_b32 s41, s44\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 9f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_waitcnt vmcnt(18)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "7:\n"  \
      "global_load_dwordx2 v[46:47], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(19)\n"  \
      "v_add_u32_dpp v96, v40, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v40, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v40, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v40, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v40, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v40, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v40, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v40, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 64f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "64:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v42, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v42, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v42, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v42, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v42, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v42, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v42, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v42, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v41, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v41, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v41, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v41, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v41, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v41, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v41, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v41, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 65f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "65:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v42, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v42, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v42, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v42, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v42, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v42, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v42, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v42, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 66f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "66:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v44, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v44, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v44, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v44, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v44, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v44, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v44, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v44, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v43, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v43, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v43, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v43, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v43, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v43, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v43, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v43, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 67f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "67:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v44, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v44, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v44, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v44, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v44, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v44, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v44, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v44, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v46, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v46, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v46, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v46, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v46, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v46, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v46, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v46, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fmac_f32_dpp %[acc0], v45, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v45, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v45, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v45, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fmac_f32_dpp %[acc1], v45, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v45, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v45, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v45, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(27)\n"  \
      "v_add_u32_dpp v96, v46, %[lane16] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v100, v46, %[lane16] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v104, v46, %[lane16] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v108, v46, %[lane16] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v112, v46, %[lane16] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v116, v46, %[lane16] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v120, v46, %[lane16] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v124, v46, %[lane16] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(22)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "s_waitcnt vmcnt(14) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fmac_f32_dpp %[acc0], v47, |v32| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc2], v47, |v33| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc4], v47, |v34| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc6], v47, |v35| row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fmac_f32_dpp %[acc1], v47, |v36| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc3], v47, |v37| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc5], v47, |v38| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "v_fmac_f32_dpp %[acc7], v47, |v39| row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_branch 7b\n"  \
      "8:\n"  \
      "9:\n"  \
      "s_waitcnt vmcnt(0) lgkmcnt(0)\n"  \
      : [acc0] "+v"(acc[0]), [acc1] "+v"(acc[1]), [acc2] "+v"(acc[2]), [acc3] "+v"(acc[3]), [acc4] "+v"(acc[4]), [acc5] "+v"(acc[5]), [acc6] "+v"(acc[6]), [acc7] "+v"(acc[7])  \
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [laneoff] "v"(laneoff), [eb] "s"(eb),  \
        [cb] "s"(cb), [bp] "s"(bp), [bstride] "s"(bstride)  \
      : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127",  \
        "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "scc", "memory")

#define STREAM4(acc, lane16, lane4, laneoff, eb, cb, bp, bstride)  \
  asm volatile(  \
      "s_load_dwordx4 s[40:43], %[cb], 0x0\n"  \
      "s_mov_b64 s[36:37], %[eb]\n"  \
      "s_mov_b64 s[38:39], %[bp]\n"  \
      "s_waitcnt lgkmcnt(0)\n"  \
      "s_mov_b32 s44, s42\n"  \
      "s_mov_b32 s42, s40\n"  \
      "s_mov_b32 s43, s41\n"  \
      "s_mov_b32 s41, s44\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 9f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "global_load_dword v48, %[lane4], s[38:39]\n"  \
      "global_load_dword v49, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v50, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v51, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 60f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "60:\n"  \
      "global_load_dword v52, %[lane4], s[38:39]\n"  \
      "global_load_dword v53, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v54, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v55, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 61f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "61:\n"  \
      "global_load_dword v56, %[lane4], s[38:39]\n"  \
      "global_load_dword v57, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v58, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v59, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 62f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "62:\n"  \
      "global_load_dword v60, %[lane4], s[38:39]\n"  \
      "global_load_dword v61, %[lane4], s[38:39] offset:256\n"  \
      "global_load_dword v62, %[lane4], s[38:39] offset:512\n"  \
      "global_load_dword v63, %[lane4], s[38:39] offset:768\n"  \
      "s_sub_u32 s40, s40, 1\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cbranch_scc0 63f\n"  \
      "s_and_b32 s40, s42, 0xff\n"  \
      "s_lshr_b64 s[42:43], s[42:43], 8\n"  \
      "s_cmp_eq_u32 s40, 0\n"  \
      "s_cselect_b32 s40, 0x7fffffff, s40\n"  \
      "s_cselect_b32 s44, 0, %[bstride]\n"  \
      "s_add_u32 s38, s38, s44\n"  \
      "s_addc_u32 s39, s39, 0\n"  \
      "63:\n"  \
      "s_waitcnt vmcnt(18)\n"  \
      "v_add_u32_dpp v64, v40, %[lane16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v68, v40, %[lane16] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v72, v40, %[lane16] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v76, v40, %[lane16] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v80, v40, %[lane16] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v84, v40, %[lane16] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v88, v40, %[lane16] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
      "v_add_u32_dpp v92, v40, %[lane16] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "7:\n"  \
      "global_load_dwordx2 v[46:47], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32 v96, v40, %[lane16]\n"  \
      "v_add_u32 v100, v40, %[lane16]\n"  \
      "v_add_u32 v104, v40, %[lane16]\n"  \
      "v_add_u32 v108, v40, %[lane16]\n"  \
      "v_add_u32 v112, v40, %[lane16]\n"  \
      "v_add_u32 v116, v40, %[lane16]\n"  \
      "v_add_u32 v120, v40, %[lane16]\n"  \
      "v_add_u32 v124, v40, %[lane16]\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(13) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32 v64, v42, %[lane16]\n"  \
      "v_add_u32 v68, v42, %[lane16]\n"  \
      "v_add_u32 v72, v42, %[lane16]\n"  \
      "v_add_u32 v76, v42, %[lane16]\n"  \
      "v_add_u32 v80, v42, %[lane16]\n"  \
      "v_add_u32 v84, v42, %[lane16]\n"  \
      "v_add_u32 v88, v42, %[lane16]\n"  \
      "v_add_u32 v92, v42, %[lane16]\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(9) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fma_f32 %[acc0], v41, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v41, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v41, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v41, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fma_f32 %[acc1], v41, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v41, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v41, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v41, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[40:41], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32 v96, v42, %[lane16]\n"  \
      "v_add_u32 v100, v42, %[lane16]\n"  \
      "v_add_u32 v104, v42, %[lane16]\n"  \
      "v_add_u32 v108, v42, %[lane16]\n"  \
      "v_add_u32 v112, v42, %[lane16]\n"  \
      "v_add_u32 v116, v42, %[lane16]\n"  \
      "v_add_u32 v120, v42, %[lane16]\n"  \
      "v_add_u32 v124, v42, %[lane16]\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(6) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32 v64, v44, %[lane16]\n"  \
      "v_add_u32 v68, v44, %[lane16]\n"  \
      "v_add_u32 v72, v44, %[lane16]\n"  \
      "v_add_u32 v76, v44, %[lane16]\n"  \
      "v_add_u32 v80, v44, %[lane16]\n"  \
      "v_add_u32 v84, v44, %[lane16]\n"  \
      "v_add_u32 v88, v44, %[lane16]\n"  \
      "v_add_u32 v92, v44, %[lane16]\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(2) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fma_f32 %[acc0], v43, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v43, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v43, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v43, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fma_f32 %[acc1], v43, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v43, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v43, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v43, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[42:43], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32 v96, v44, %[lane16]\n"  \
      "v_add_u32 v100, v44, %[lane16]\n"  \
      "v_add_u32 v104, v44, %[lane16]\n"  \
      "v_add_u32 v108, v44, %[lane16]\n"  \
      "v_add_u32 v112, v44, %[lane16]\n"  \
      "v_add_u32 v116, v44, %[lane16]\n"  \
      "v_add_u32 v120, v44, %[lane16]\n"  \
      "v_add_u32 v124, v44, %[lane16]\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v48\n"  \
      "v_sub_f32 v33, v65, v49\n"  \
      "v_sub_f32 v34, v66, v50\n"  \
      "v_sub_f32 v35, v67, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v48\n"  \
      "v_sub_f32 v37, v69, v49\n"  \
      "v_sub_f32 v38, v70, v50\n"  \
      "v_sub_f32 v39, v71, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v48\n"  \
      "v_sub_f32 v33, v73, v49\n"  \
      "v_sub_f32 v34, v74, v50\n"  \
      "v_sub_f32 v35, v75, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v48\n"  \
      "v_sub_f32 v37, v77, v49\n"  \
      "v_sub_f32 v38, v78, v50\n"  \
      "v_sub_f32 v39, v79, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v48\n"  \
      "v_sub_f32 v33, v81, v49\n"  \
      "v_sub_f32 v34, v82, v50\n"  \
      "v_sub_f32 v35, v83, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v48\n"  \
      "v_sub_f32 v37, v85, v49\n"  \
      "v_sub_f32 v38, v86, v50\n"  \
      "v_sub_f32 v39, v87, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v48\n"  \
      "v_sub_f32 v33, v89, v49\n"  \
      "v_sub_f32 v34, v90, v50\n"  \
      "v_sub_f32 v35, v91, v51\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v48\n"  \
      "v_sub_f32 v37, v93, v49\n"  \
      "v_sub_f32 v38, v94, v50\n"  \
      "v_sub_f32 v39, v95, v51\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32 v64, v46, %[lane16]\n"  \
      "v_add_u32 v68, v46, %[lane16]\n"  \
      "v_add_u32 v72, v46, %[lane16]\n"  \
      "v_add_u32 v76, v46, %[lane16]\n"  \
      "v_add_u32 v80, v46, %[lane16]\n"  \
      "v_add_u32 v84, v46, %[lane16]\n"  \
      "v_add_u32 v88, v46, %[lane16]\n"  \
      "v_add_u32 v92, v46, %[lane16]\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v52\n"  \
      "v_sub_f32 v33, v97, v53\n"  \
      "v_sub_f32 v34, v98, v54\n"  \
      "v_sub_f32 v35, v99, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v52\n"  \
      "v_sub_f32 v37, v101, v53\n"  \
      "v_sub_f32 v38, v102, v54\n"  \
      "v_sub_f32 v39, v103, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v52\n"  \
      "v_sub_f32 v33, v105, v53\n"  \
      "v_sub_f32 v34, v106, v54\n"  \
      "v_sub_f32 v35, v107, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v52\n"  \
      "v_sub_f32 v37, v109, v53\n"  \
      "v_sub_f32 v38, v110, v54\n"  \
      "v_sub_f32 v39, v111, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v52\n"  \
      "v_sub_f32 v33, v113, v53\n"  \
      "v_sub_f32 v34, v114, v54\n"  \
      "v_sub_f32 v35, v115, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v52\n"  \
      "v_sub_f32 v37, v117, v53\n"  \
      "v_sub_f32 v38, v118, v54\n"  \
      "v_sub_f32 v39, v119, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v52\n"  \
      "v_sub_f32 v33, v121, v53\n"  \
      "v_sub_f32 v34, v122, v54\n"  \
      "v_sub_f32 v35, v123, v55\n"  \
      "v_fma_f32 %[acc0], v45, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v45, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v45, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v45, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v52\n"  \
      "v_sub_f32 v37, v125, v53\n"  \
      "v_sub_f32 v38, v126, v54\n"  \
      "v_sub_f32 v39, v127, v55\n"  \
      "v_fma_f32 %[acc1], v45, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v45, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v45, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v45, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "global_load_dwordx2 v[44:45], %[laneoff], s[36:37]\n"  \
      "s_add_u32 s36, s36, 0x80\n"  \
      "s_addc_u32 s37, s37, 0\n"  \
      "s_waitcnt vmcnt(3)\n"  \
      "v_add_u32 v96, v46, %[lane16]\n"  \
      "v_add_u32 v100, v46, %[lane16]\n"  \
      "v_add_u32 v104, v46, %[lane16]\n"  \
      "v_add_u32 v108, v46, %[lane16]\n"  \
      "v_add_u32 v112, v46, %[lane16]\n"  \
      "v_add_u32 v116, v46, %[lane16]\n"  \
      "v_add_u32 v120, v46, %[lane16]\n"  \
      "v_add_u32 v124, v46, %[lane16]\n"  \
      "ds_read_b128 v[96:99], v96\n"  \
      "ds_read_b128 v[100:103], v100\n"  \
      "ds_read_b128 v[104:107], v104\n"  \
      "ds_read_b128 v[108:111], v108\n"  \
      "ds_read_b128 v[112:115], v112\n"  \
      "ds_read_b128 v[116:119], v116\n"  \
      "ds_read_b128 v[120:123], v120\n"  \
      "ds_read_b128 v[124:127], v124\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v64, v56\n"  \
      "v_sub_f32 v33, v65, v57\n"  \
      "v_sub_f32 v34, v66, v58\n"  \
      "v_sub_f32 v35, v67, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v68, v56\n"  \
      "v_sub_f32 v37, v69, v57\n"  \
      "v_sub_f32 v38, v70, v58\n"  \
      "v_sub_f32 v39, v71, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v72, v56\n"  \
      "v_sub_f32 v33, v73, v57\n"  \
      "v_sub_f32 v34, v74, v58\n"  \
      "v_sub_f32 v35, v75, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v76, v56\n"  \
      "v_sub_f32 v37, v77, v57\n"  \
      "v_sub_f32 v38, v78, v58\n"  \
      "v_sub_f32 v39, v79, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v80, v56\n"  \
      "v_sub_f32 v33, v81, v57\n"  \
      "v_sub_f32 v34, v82, v58\n"  \
      "v_sub_f32 v35, v83, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v84, v56\n"  \
      "v_sub_f32 v37, v85, v57\n"  \
      "v_sub_f32 v38, v86, v58\n"  \
      "v_sub_f32 v39, v87, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v88, v56\n"  \
      "v_sub_f32 v33, v89, v57\n"  \
      "v_sub_f32 v34, v90, v58\n"  \
      "v_sub_f32 v35, v91, v59\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v92, v56\n"  \
      "v_sub_f32 v37, v93, v57\n"  \
      "v_sub_f32 v38, v94, v58\n"  \
      "v_sub_f32 v39, v95, v59\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_waitcnt vmcnt(2)\n"  \
      "v_add_u32 v64, v40, %[lane16]\n"  \
      "v_add_u32 v68, v40, %[lane16]\n"  \
      "v_add_u32 v72, v40, %[lane16]\n"  \
      "v_add_u32 v76, v40, %[lane16]\n"  \
      "v_add_u32 v80, v40, %[lane16]\n"  \
      "v_add_u32 v84, v40, %[lane16]\n"  \
      "v_add_u32 v88, v40, %[lane16]\n"  \
      "v_add_u32 v92, v40, %[lane16]\n"  \
      "ds_read_b128 v[64:67], v64\n"  \
      "ds_read_b128 v[68:71], v68\n"  \
      "ds_read_b128 v[72:75], v72\n"  \
      "ds_read_b128 v[76:79], v76\n"  \
      "ds_read_b128 v[80:83], v80\n"  \
      "ds_read_b128 v[84:87], v84\n"  \
      "ds_read_b128 v[88:91], v88\n"  \
      "ds_read_b128 v[92:95], v92\n"  \
      "s_waitcnt vmcnt(63) lgkmcnt(8)\n"  \
      "v_sub_f32 v32, v96, v60\n"  \
      "v_sub_f32 v33, v97, v61\n"  \
      "v_sub_f32 v34, v98, v62\n"  \
      "v_sub_f32 v35, v99, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v100, v60\n"  \
      "v_sub_f32 v37, v101, v61\n"  \
      "v_sub_f32 v38, v102, v62\n"  \
      "v_sub_f32 v39, v103, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v104, v60\n"  \
      "v_sub_f32 v33, v105, v61\n"  \
      "v_sub_f32 v34, v106, v62\n"  \
      "v_sub_f32 v35, v107, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v108, v60\n"  \
      "v_sub_f32 v37, v109, v61\n"  \
      "v_sub_f32 v38, v110, v62\n"  \
      "v_sub_f32 v39, v111, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v112, v60\n"  \
      "v_sub_f32 v33, v113, v61\n"  \
      "v_sub_f32 v34, v114, v62\n"  \
      "v_sub_f32 v35, v115, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v116, v60\n"  \
      "v_sub_f32 v37, v117, v61\n"  \
      "v_sub_f32 v38, v118, v62\n"  \
      "v_sub_f32 v39, v119, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "v_sub_f32 v32, v120, v60\n"  \
      "v_sub_f32 v33, v121, v61\n"  \
      "v_sub_f32 v34, v122, v62\n"  \
      "v_sub_f32 v35, v123, v63\n"  \
      "v_fma_f32 %[acc0], v47, |v32|, %[acc0]\n"  \
      "v_fma_f32 %[acc2], v47, |v33|, %[acc2]\n"  \
      "v_fma_f32 %[acc4], v47, |v34|, %[acc4]\n"  \
      "v_fma_f32 %[acc6], v47, |v35|, %[acc6]\n"  \
      "v_sub_f32 v36, v124, v60\n"  \
      "v_sub_f32 v37, v125, v61\n"  \
      "v_sub_f32 v38, v126, v62\n"  \
      "v_sub_f32 v39, v127, v63\n"  \
      "v_fma_f32 %[acc1], v47, |v36|, %[acc1]\n"  \
      "v_fma_f32 %[acc3], v47, |v37|, %[acc3]\n"  \
      "v_fma_f32 %[acc5], v47, |v38|, %[acc5]\n"  \
      "v_fma_f32 %[acc7], v47, |v39|, %[acc7]\n"  \
      "s_sub_u32 s41, s41, 1\n"  \
      "s_cmp_eq_u32 s41, 0\n"  \
      "s_cbranch_scc1 8f\n"  \
      "s_branch 7b\n"  \
      "8:\n"  \
      "9:\n"  \
      "s_waitcnt vmcnt(0) lgkmcnt(0)\n"  \
      : [acc0] "+v"(acc[0]), [acc1] "+v"(acc[1]), [acc2] "+v"(acc[2]), [acc3] "+v"(acc[3]), [acc4] "+v"(acc[4]), [acc5] "+v"(acc[5]), [acc6] "+v"(acc[6]), [acc7] "+v"(acc[7])  \
      : [lane16] "v"(lane16), [lane4] "v"(lane4), [laneoff] "v"(laneoff), [eb] "s"(eb),  \
        [cb] "s"(cb), [bp] "s"(bp), [bstride] "s"(bstride)  \
      : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127",  \
        "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "scc", "memory")


constexpr int kTile = 128, kSWaves = 16, kStreamGroups = 128;
template <int V>
__global__ __launch_bounds__(1024) void kern(const uint2* ent, const uint4* cnt, const float* xs, int PW, int ntiles,
                                             int tiles_per_wg, float* out) {
  __shared__ float4 As[kTile * 64];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int r = wave; r < kTile; r += kSWaves) As[r * 64 + lane] = make_float4(r * 0.01f + lane, r * 0.01f + lane + 1, r * 0.01f + lane + 2, r * 0.01f + lane + 3);
  __syncthreads();
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t lane16 = (uint32_t)(uintptr_t)As + lane * 16u, lane4 = lane * 4u, laneoff = (lane & 15) * 8u;
  const uint32_t bstride = kSWaves * PW * 4;
  for (int k = 0; k < tiles_per_wg; k++) {
    const int t = __builtin_amdgcn_readfirstlane((int)((blockIdx.x / 32 * tiles_per_wg + k) % ntiles));
    const int64_t st = (int64_t)t * kSWaves + wave;
    const uint64_t eb = (uint64_t)(uintptr_t)(ent + st * kStreamGroups * 8);
    const uint64_t cb = (uint64_t)(uintptr_t)(cnt + st);
    const uint64_t bp = (uint64_t)(uintptr_t)(xs + (int64_t)wave * PW);
    if (V == 0) STREAM(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 1) STREAM1(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 2) STREAM2(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 3) STREAM3(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
    if (V == 4) STREAM4(acc, lane16, lane4, laneoff, eb, cb, bp, bstride);
  }
  for (int i = 0; i < 8; i++) out[((size_t)blockIdx.x * 1024 + threadIdx.x) * 8 + i] = acc[i];
}

int main() {
  const int ntiles = 2048, PW = 1024;
  const double dens = 0.42;
  std::mt19937 rng(1);
  std::vector<uint2> ent((size_t)(ntiles + 1) * kSWaves * kStreamGroups * 8, make_uint2(0, 0));
  std::vector<uint4> cnt((size_t)(ntiles + 1) * kSWaves, make_uint4(0, 0, 0, 0));
  std::vector<int64_t> tile_groups(ntiles, 0);
  for (int t = 0; t < ntiles; t++)
    for (int w = 0; w < kSWaves; w++) {
      const int64_t st = (int64_t)t * kSWaves + w;
      uint2* o = &ent[st * kStreamGroups * 8];
      int off = 0, tot = 0;
      uint32_t c03 = 0, c47 = 0;
      for (int m = 0; m < kTile / kSWaves; m++) {
        int c = 0;
        for (int ii = 0; ii < kTile; ii++)
          if (std::uniform_real_distribution<double>(0, 1)(rng) < dens)
            o[off + c++] = make_uint2(ii * 1024u, __builtin_bit_cast(uint32_t, (float)(1 + (ii + m) % 7) * 0.125f));
        int pad = c == 0 ? 8 : (c + 7) / 8 * 8;
        for (int e = c; e < pad; e++) o[off + e] = make_uint2(0, 0);
        off += pad;
        const int ng = pad / 8;
        if (m < 4) c03 |= (uint32_t)ng << (8 * m); else c47 |= (uint32_t)ng << (8 * (m - 4));
        tot += ng;
      }
      cnt[st] = make_uint4(c03, c47, (uint32_t)tot, 0);
      tile_groups[t] += tot;
    }
  uint2* dent; uint4* dcnt; float *dxs, *dout;
  CHK(hipMalloc(&dent, ent.size() * 8)); CHK(hipMemcpy(dent, ent.data(), ent.size() * 8, hipMemcpyHostToDevice));
  CHK(hipMalloc(&dcnt, cnt.size() * 16)); CHK(hipMemcpy(dcnt, cnt.data(), cnt.size() * 16, hipMemcpyHostToDevice));
  // B rows: xs[row][f0 + lane + 64 f] = 0.5 * f (row-independent)
  std::vector<float> hx((size_t)(kTile + 2) * PW);
  for (size_t i = 0; i < hx.size(); i++) hx[i] = 0.5f * (float)((i % PW) / 64 % 4);
  CHK(hipMalloc(&dxs, hx.size() * 4)); CHK(hipMemcpy(dxs, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  const int wgs = 4096, tpw = 4;
  CHK(hipMalloc(&dout, (size_t)wgs * 1024 * 8 * 4));
  // correctness on a few workgroups
  kern<0><<<wgs, 1024>>>(dent, dcnt, dxs, PW, ntiles, tpw, dout);
  CHK(hipDeviceSynchronize());
  std::vector<float> ho((size_t)wgs * 1024 * 8);
  CHK(hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0; double maxrel = 0;
  for (int b = 0; b < wgs; b += 397)
    for (int w = 0; w < kSWaves; w++)
      for (int lane = 0; lane < 64; lane += 7) {
        double want[4] = {0, 0, 0, 0}, got[4] = {0, 0, 0, 0};
        for (int k = 0; k < tpw; k++) {
          const int t = (b / 32 * tpw + k) % ntiles;
          const int64_t st = (int64_t)t * kSWaves + w;
          const uint2* o = &ent[st * kStreamGroups * 8];
          for (int e = 0; e < (int)cnt[st].z * 8; e++) {
            const int r = o[e].x / 1024; const float wt = __builtin_bit_cast(float, o[e].y);
            for (int f = 0; f < 4; f++) want[f] += wt * fabs((r * 0.01f + lane + f) - 0.5 * f);
          }
        }
        const float* g = &ho[((size_t)b * 1024 + w * 64 + lane) * 8];
        for (int f = 0; f < 4; f++) {
          got[f] = (double)g[2 * f] + g[2 * f + 1];
          const double rel = fabs(got[f] - want[f]) / fmax(1.0, fabs(want[f]));
          if (rel > maxrel) maxrel = rel;
          if (rel > 1e-4) { if (bad < 5) printf("mismatch wg %d wave %d lane %d f %d: got %g want %g\n", b, w, lane, f, got[f], want[f]); bad++; }
        }
      }
  printf("check: %s (max rel err %.2e)\n", bad ? "WRONG" : "ok", maxrel);
  fflush(stdout);
  double g_total = 0;
  for (int b = 0; b < wgs; b++) for (int k = 0; k < tpw; k++) g_total += tile_groups[(b / 32 * tpw + k) % ntiles];
  const char* nm[5] = {"dpp stream", "plain fma", "no per-group B", "no LDS reads", "plain fma+add, no B"};
  for (int v = 0; v < 5; v++) {
  auto K = v == 0 ? kern<0> : v == 1 ? kern<1> : v == 2 ? kern<2> : v == 3 ? kern<3> : kern<4>;
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; rep++) {
    CHK(hipEventRecord(e0));
    K<<<wgs, 1024>>>(dent, dcnt, dxs, PW, ntiles, tpw, dout);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep && ms < best) best = ms;
  }
  const double valu_ms = g_total * 72 * 2 / 1024.0 / 2.4e9 * 1e3;
  printf("%-22s %8.3f ms   groups %.3g  cycles/group/SIMD %.1f  per entry-feature %.2f  (VALU floor %.3f ms = %.0f%%)\n",
         nm[v], best, g_total, best * 1e-3 * 2.4e9 * 1024 / g_total, best * 1e-3 * 2.4e9 * 1024 / g_total / 32, valu_ms, 100 * valu_ms / best);
  fflush(stdout);
  }
  return 0;
}
