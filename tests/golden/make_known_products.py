"""Writes known_products.json: hand-computed known answers of indexed expressions.

The input values and expected outputs are the known-answer data of the reference's unit tests
(cited per case as file:line under src/unitTests/); the expression cases are re-expressed in the
token notation of oracle/indexed.py. Run: python tests/golden/make_known_products.py
"""
import json
import os

A2 = {"dims": [2, 2], "values": [1, 2, 3, 4]}
B2 = {"dims": [2, 2], "values": [5, 6, 7, 8]}
V2a = {"dims": [2], "values": [1, 2]}
V2b = {"dims": [2], "values": [3, 4]}
V3 = {"dims": [3], "values": [5, 6, 7]}
A12 = {"dims": [1, 2], "values": [1, 2]}
B23 = {"dims": [2, 3], "values": [3, 4, 5, 6, 7, 8]}
TA = {"dims": [2, 2], "values": [1, 2, 4, 8]}
TB = {"dims": [2, 2, 2], "values": [1, 2, 4, 8, 16, 32, 64, 128]}
TC = {"dims": [2, 2, 2, 2], "values": [2 ** k for k in range(16)]}
R24 = {"dims": [2, 2, 3, 1, 2], "values": list(range(1, 25))}
ID24 = list(range(1, 25))
SW24 = [1, 2, 3, 4, 5, 6, 13, 14, 15, 16, 17, 18, 7, 8, 9, 10, 11, 12, 19, 20, 21, 22, 23, 24]


def case(name, src, inputs, lhs, rhs, expected, scale=1.0):
    return {"name": name, "source": src, "inputs": inputs, "lhs": lhs, "rhs": rhs, "scale": scale, "expected": expected}


CASES = [
    case("order0", "fullTensor_product.cxx:30-40", {"A": {"dims": [], "values": [42]}, "B": {"dims": [], "values": [73]}},
         [], [["A", []], ["B", []]], [42 * 73]),
    case("outer_ij", "fullTensor_product.cxx:63-64", {"A": V2a, "B": V2b}, ["i", "j"], [["A", ["i"]], ["B", ["j"]]], [3, 4, 6, 8]),
    case("outer_ji", "fullTensor_product.cxx:67-68", {"A": V2a, "B": V2b}, ["i", "j"], [["A", ["j"]], ["B", ["i"]]], [3, 6, 4, 8]),
    case("inner", "fullTensor_product.cxx:73-74", {"A": V2a, "B": V2b}, [], [["A", ["i"]], ["B", ["i"]]], [11]),
    case("outer_diff", "fullTensor_product.cxx:78-79", {"A": V2a, "C": V3}, ["i", "j"], [["A", ["i"]], ["C", ["j"]]],
         [5, 6, 7, 10, 12, 14]),
    case("outer_diff_T", "fullTensor_product.cxx:82-83", {"A": V2a, "C": V3}, ["i", "j"], [["C", ["i"]], ["A", ["j"]]],
         [5, 10, 6, 12, 7, 14]),
    case("o2_ijkl", "fullTensor_product.cxx:120-121", {"A": A2, "B": B2}, ["i", "j", "k", "l"], [["A", ["i", "j"]], ["B", ["k", "l"]]],
         [5, 6, 7, 8, 10, 12, 14, 16, 15, 18, 21, 24, 20, 24, 28, 32]),
    case("o2_swap_pairs", "fullTensor_product.cxx:124-125", {"A": A2, "B": B2}, ["i", "j", "k", "l"],
         [["A", ["k", "l"]], ["B", ["i", "j"]]], [5, 10, 15, 20, 6, 12, 18, 24, 7, 14, 21, 28, 8, 16, 24, 32]),
    case("o2_ji", "fullTensor_product.cxx:130-131", {"A": A2, "B": B2}, ["i", "j", "k", "l"], [["A", ["j", "i"]], ["B", ["k", "l"]]],
         [5, 6, 7, 8, 15, 18, 21, 24, 10, 12, 14, 16, 20, 24, 28, 32]),
    case("o2_lk", "fullTensor_product.cxx:134-135", {"A": A2, "B": B2}, ["i", "j", "k", "l"], [["A", ["i", "j"]], ["B", ["l", "k"]]],
         [5, 7, 6, 8, 10, 14, 12, 16, 15, 21, 18, 24, 20, 28, 24, 32]),
    case("o2_lj_ki", "fullTensor_product.cxx:140-141", {"A": A2, "B": B2}, ["i", "j", "k", "l"],
         [["A", ["l", "j"]], ["B", ["k", "i"]]], [5, 15, 7, 21, 10, 20, 14, 28, 6, 18, 8, 24, 12, 24, 16, 32]),
    case("o2_ik_jl", "fullTensor_product.cxx:144-145", {"A": A2, "B": B2}, ["i", "j", "k", "l"],
         [["A", ["i", "k"]], ["B", ["j", "l"]]], [5, 6, 10, 12, 7, 8, 14, 16, 15, 18, 20, 24, 21, 24, 28, 32]),
    case("o2_kj_il", "fullTensor_product.cxx:150-151", {"A": A2, "B": B2}, ["i", "j", "k", "l"],
         [["A", ["k", "j"]], ["B", ["i", "l"]]], [5, 6, 15, 18, 10, 12, 20, 24, 7, 8, 21, 24, 14, 16, 28, 32]),
    case("o2_il_kj", "fullTensor_product.cxx:154-155", {"A": A2, "B": B2}, ["i", "j", "k", "l"],
         [["A", ["i", "l"]], ["B", ["k", "j"]]], [5, 10, 7, 14, 6, 12, 8, 16, 15, 20, 21, 28, 18, 24, 24, 32]),
    case("o2_span2", "fullTensor_product.cxx:160-161", {"A": A2, "B": B2}, ["i^2", "j^2"], [["A", ["i^2"]], ["B", ["j^2"]]],
         [5, 6, 7, 8, 10, 12, 14, 16, 15, 18, 21, 24, 20, 24, 28, 32]),
    case("o2_span2_swap", "fullTensor_product.cxx:164-165", {"A": A2, "B": B2}, ["i^2", "j^2"], [["A", ["j^2"]], ["B", ["i^2"]]],
         [5, 10, 15, 20, 6, 12, 18, 24, 7, 14, 21, 28, 8, 16, 24, 32]),
    case("mm_ij_jk", "fullTensor_product.cxx:172-173", {"A": A2, "B": B2}, ["i", "k"], [["A", ["i", "j"]], ["B", ["j", "k"]]],
         [19, 22, 43, 50]),
    case("mm_ji_jk", "fullTensor_product.cxx:174-175", {"A": A2, "B": B2}, ["i", "k"], [["A", ["j", "i"]], ["B", ["j", "k"]]],
         [26, 30, 38, 44]),
    case("mm_ij_kj", "fullTensor_product.cxx:176-177", {"A": A2, "B": B2}, ["i", "k"], [["A", ["i", "j"]], ["B", ["k", "j"]]],
         [17, 23, 39, 53]),
    case("mm_ji_kj", "fullTensor_product.cxx:178-179", {"A": A2, "B": B2}, ["i", "k"], [["A", ["j", "i"]], ["B", ["k", "j"]]],
         [23, 31, 34, 46]),
    case("mm_ij_jk_T", "fullTensor_product.cxx:181-182", {"A": A2, "B": B2}, ["k", "i"], [["A", ["i", "j"]], ["B", ["j", "k"]]],
         [19, 43, 22, 50]),
    case("mm_ji_kj_T", "fullTensor_product.cxx:187-188", {"A": A2, "B": B2}, ["k", "i"], [["A", ["j", "i"]], ["B", ["k", "j"]]],
         [23, 34, 31, 46]),
    case("full_ij_ij", "fullTensor_product.cxx:191-192", {"A": A2, "B": B2}, [], [["A", ["i", "j"]], ["B", ["i", "j"]]], [70]),
    case("full_ij_ji", "fullTensor_product.cxx:193-194", {"A": A2, "B": B2}, [], [["A", ["i", "j"]], ["B", ["j", "i"]]], [69]),
    case("full_span2", "fullTensor_product.cxx:197-198", {"A": A2, "B": B2}, [], [["A", ["i^2"]], ["B", ["i^2"]]], [70]),
    case("diff_outer", "fullTensor_product.cxx:224-225", {"A": A12, "B": B23}, ["i", "j", "k", "l"],
         [["A", ["i", "j"]], ["B", ["k", "l"]]], [3, 4, 5, 6, 7, 8, 6, 8, 10, 12, 14, 16]),
    case("diff_outer_ik", "fullTensor_product.cxx:226-227", {"A": A12, "B": B23}, ["i", "j", "k", "l"],
         [["A", ["i", "k"]], ["B", ["j", "l"]]], [3, 4, 5, 6, 8, 10, 6, 7, 8, 12, 14, 16]),
    case("diff_mm", "fullTensor_product.cxx:232-233", {"A": A12, "B": B23}, ["i", "k"], [["A", ["i", "j"]], ["B", ["j", "k"]]],
         [15, 18, 21]),
    case("diff_mm_rev", "fullTensor_product.cxx:236-237", {"A": A12, "B": B23}, ["i", "k"], [["B", ["j", "k"]], ["A", ["i", "j"]]],
         [15, 18, 21]),
    case("trace_A", "fullTensor_trace.cxx:70-71", {"A": TA}, [], [["A", ["i", "i"]]], [9]),
    case("trace_B_iij", "fullTensor_trace.cxx:73-74", {"B": TB}, ["j"], [["B", ["i", "i", "j"]]], [65, 130]),
    case("trace_B_iji", "fullTensor_trace.cxx:75-76", {"B": TB}, ["j"], [["B", ["i", "j", "i"]]], [33, 132]),
    case("trace_B_jii", "fullTensor_trace.cxx:77-78", {"B": TB}, ["j"], [["B", ["j", "i", "i"]]], [9, 144]),
    case("trace_C_iijk", "fullTensor_trace.cxx:80-81", {"C": TC}, ["j", "k"], [["C", ["i", "i", "j", "k"]]], [4097, 8194, 16388, 32776]),
    case("trace_C_ijik", "fullTensor_trace.cxx:82-83", {"C": TC}, ["j", "k"], [["C", ["i", "j", "i", "k"]]], [1025, 2050, 16400, 32800]),
    case("trace_C_ijki", "fullTensor_trace.cxx:84-85", {"C": TC}, ["j", "k"], [["C", ["i", "j", "k", "i"]]], [513, 2052, 8208, 32832]),
    case("trace_C_jiik", "fullTensor_trace.cxx:86-87", {"C": TC}, ["j", "k"], [["C", ["j", "i", "i", "k"]]], [65, 130, 16640, 33280]),
    case("trace_C_jiki", "fullTensor_trace.cxx:88-89", {"C": TC}, ["j", "k"], [["C", ["j", "i", "k", "i"]]], [33, 132, 8448, 33792]),
    case("trace_C_jkii", "fullTensor_trace.cxx:90-91", {"C": TC}, ["j", "k"], [["C", ["j", "k", "i", "i"]]], [9, 144, 2304, 36864]),
    case("trace_C_iijk_T", "fullTensor_trace.cxx:93-94", {"C": TC}, ["k", "j"], [["C", ["i", "i", "j", "k"]]],
         [4097, 16388, 8194, 32776]),
    case("trace_C_jkii_T", "fullTensor_trace.cxx:103-104", {"C": TC}, ["k", "j"], [["C", ["j", "k", "i", "i"]]],
         [9, 2304, 144, 36864]),
    case("trace_fixed_0", "fullTensor_trace.cxx:106-107", {"C": TC}, ["k"], [["C", [0, "k", "i", "i"]]], [9, 144]),
    case("trace_fixed_1", "fullTensor_trace.cxx:108-109", {"C": TC}, ["k"], [["C", [1, "k", "i", "i"]]], [2304, 36864]),
    case("trace_fixed_mid0", "fullTensor_trace.cxx:110-111", {"C": TC}, ["j"], [["C", ["j", 0, "i", "i"]]], [9, 2304]),
    case("trace_fixed_mid1", "fullTensor_trace.cxx:112-113", {"C": TC}, ["j"], [["C", ["j", 1, "i", "i"]]], [144, 36864]),
    case("trace_double_iijj", "fullTensor_trace.cxx:115-116", {"C": TC}, [], [["C", ["i", "i", "j", "j"]]], [1 + 8 + 4096 + 32768]),
    case("trace_double_ijij", "fullTensor_trace.cxx:117-118", {"C": TC}, [], [["C", ["i", "j", "i", "j"]]], [1 + 32 + 1024 + 32768]),
    case("trace_double_ijji", "fullTensor_trace.cxx:119-120", {"C": TC}, [], [["C", ["i", "j", "j", "i"]]], [1 + 64 + 512 + 32768]),
    case("assign_identity", "fullTensor_assignment.cxx:54-55", {"A": R24}, ["i", "j", "k", "l", "m"],
         [["A", ["i", "j", "k", "l", "m"]]], ID24),
    case("assign_all_but_0", "fullTensor_assignment.cxx:56-57", {"A": R24}, ["i&0"], [["A", ["i&0"]]], ID24),
    case("assign_span5", "fullTensor_assignment.cxx:58-59", {"A": R24}, ["i&0"], [["A", ["i^5"]]], ID24),
    case("assign_mixed_spans", "fullTensor_assignment.cxx:62-63", {"A": R24}, ["i^3", "j&3"], [["A", ["i&2", "j^2"]]], ID24),
    case("assign_swap", "fullTensor_assignment.cxx:67-68", {"A": R24}, ["i", "j", "k", "l", "m"],
         [["A", ["j", "i", "k", "l", "m"]]], SW24),
    case("assign_swap_lhs", "fullTensor_assignment.cxx:69-70", {"A": R24}, ["j", "i", "k", "l", "m"],
         [["A", ["i", "j", "k", "l", "m"]]], SW24),
    case("assign_ikj", "fullTensor_assignment.cxx:72-73", {"A": R24}, ["i", "k", "j", "l", "m"],
         [["A", ["i", "j", "k", "l", "m"]]], [1, 2, 7, 8, 3, 4, 9, 10, 5, 6, 11, 12, 13, 14, 19, 20, 15, 16, 21, 22, 17, 18, 23, 24]),
    case("assign_unit_mode_swap", "fullTensor_assignment.cxx:77-78", {"A": R24}, ["i", "j", "k", "l", "m"],
         [["A", ["i", "j", "l", "k", "m"]]], ID24),
]

# expressions the reference rejects with misc::generic_error (indices.cxx:28-78)
ERRORS = [
    {"name": "span_too_large", "source": "indices.cxx:33", "dims": [10, 10], "lhs": ["i", "j^2"], "rhs": [["A", ["j^2", "i"]]]},
    {"name": "inverse_span_too_large", "source": "indices.cxx:43", "dims": [10, 10], "lhs": ["i", "j"], "rhs": [["A", ["j", "i&0"]]]},
    {"name": "fractional_span_too_large", "source": "indices.cxx:53", "dims": [10, 10], "lhs": ["i", "j"], "rhs": [["A", ["j", "i/1"]]]},
    {"name": "fractional_span_not_dividing", "source": "indices.cxx:63", "dims": [10, 10], "lhs": ["i", "j"],
     "rhs": [["A", ["j", "i/3"]]]},
    {"name": "lhs_index_contracted", "source": "indices.cxx:71-72", "dims": [10, 10], "dims_b": [10], "lhs": ["j"],
     "rhs": [["A", ["i", "j"]], ["B", ["j"]]]},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "known_products.json")
    with open(out, "w") as f:
        json.dump({"cases": CASES, "errors": ERRORS}, f, indent=1)
    print(f"wrote {len(CASES)} cases and {len(ERRORS)} error cases to {out}")
