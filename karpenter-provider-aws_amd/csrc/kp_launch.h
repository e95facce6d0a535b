// kp_launch.h — device view of a launch-selection batch (kp_launch_select; filter.go chain + Truncate +
// getCapacityType + the offering side of getOverrides).  Shared by kp_host.cpp and kp_launch.hip.
#pragma once
#include <stdint.h>

#define KL_MAX_OFF 64        // offerings per instance type (u64 masks)
#define KL_MAX_SUB 4         // sub-batches of one kp_launch_select call (host / device pipeline)
#define KL_ROLES 5           // offering requirement keys: zone, capacity-type, zone-id, reservation-id, reservation-type
#define KL_ROLE_ZONE 0
#define KL_ROLE_CT 1
#define KL_ROLE_ZONEID 2
#define KL_ROLE_RESVID 3
#define KL_ROLE_RESVTYPE 4

// offering role value: >= 0 dictionary value id, or
#define KL_V_ABSENT (-1)     // key absent from Offering.Requirements
#define KL_V_DNE (-2)        // DoesNotExist

// request key entry flags
#define KLK_SINGLE 1u        // catalog key with single-valued types (type_val)
#define KLK_MULTI 2u         // multi-valued catalog key (multi_mask, <= 64 values)
#define KLK_DNE_OK 4u        // request operator NotIn / DoesNotExist (Intersects exception for a DoesNotExist type)

// offering role modes
#define KLR_PASS 0           // request does not constrain the key; an In offering passes (well-known key)
#define KLR_FAIL_IN 1        // request does not constrain the key; an In offering fails (not well-known)
#define KLR_CONSTRAINED 2    // bit test against the request's value bitset (DoesNotExist per KLK_DNE_OK)

struct KlKey {               // one catalog key the request constrains / must leave undefined
    int32_t k;               // catalog key (row of type_val / dne_mask)
    int32_t mi;              // multi index (KLK_MULTI) or -1
    uint32_t flags;
    int32_t woff;            // word offset of the value bitset in KpLaunch.words
};

struct KlRole {
    int32_t mode;            // KLR_*
    uint32_t flags;          // KLK_DNE_OK
    int32_t woff;
    int32_t pad;
};

struct KlMinKey {            // SatisfiesMinValues: distinct values of key k among the truncated types >= minv
    int32_t k, mi, nvals, minv;
};

struct KlReq {
    int32_t key_off, n_keys;         // constrained keys (KlKey)
    int32_t und_off, n_und;          // unconstrained keys that are not well-known: an In type fails (KlKey)
    int32_t min_off, n_min;          // minValues keys (KlMinKey)
    int32_t has_min;                 // Requirements.HasMinValues()
    int32_t ct_has[3];               // Get(capacity-type).Has(on-demand / spot / reserved)
    KlRole role[KL_ROLES];
};

struct KpLaunch {
    // catalog
    int T, TW, R, M;                 // M = max_instance_types
    const uint16_t* type_val;        // [Kc][T]
    const uint64_t* multi_mask;      // [n_multi][T]
    const uint64_t* dne_mask;        // [Kc][TW]
    const int64_t* alloc;            // [R][T]
    const uint32_t* name_rank;       // [T]
    const uint8_t* exotic;           // [T] metal size or accelerator capacity (filter.go:294-312)
    const int32_t* off_begin;        // [T+1] offering rows grouped by type
    const int32_t* off_val;          // [KL_ROLES][O]
    const int32_t* ct_code;          // [O] KP_CT_* of the offering
    const int32_t* rt_code;          // [O] reservation type: -1 none, 0 default, 1 capacity-block
    const double* off_price;         // [O]
    const uint8_t* off_avail;        // [O]
    const int32_t* off_rcap;         // [O] ReservationCapacity
    // requests
    int L;
    const KlReq* req;                // [L]
    const KlKey* keys;
    const KlMinKey* mins;
    const uint64_t* words;
    const int64_t* requests;         // [L][R]
    // outputs (fixed stride)
    int32_t* out_hdr;                // [L][8 + KP_N_FILTERS]: status, failed, ct, n_types, n_over, n_options, -, -, rejected
    int32_t* out_types;              // [L][M]
    uint64_t* out_over;              // [L][M] override offering mask per kept slot (bit j = row off_begin[t] + j)
};

#define KL_HDR 14
