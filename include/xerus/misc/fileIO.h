// xerus data files (reference include/xerus/misc/fileIO.h:103-163): "Xerus <type> datafile." header,
// BINARY or TSV stream of the object (xerus_amd/csrc/host/fileio.cpp).
#pragma once
#include <string>

#include "../tensor.h"
#include "../tensorNetwork.h"
#include "../ttNetwork.h"

namespace xerus {
namespace misc {
void save_to_file(const Tensor& _tensor, const std::string& _filename, const FileFormat _format = FileFormat::BINARY);
void save_to_file(const TensorNetwork& _network, const std::string& _filename, const FileFormat _format = FileFormat::BINARY);
void save_to_file(const TTTensor& _tt, const std::string& _filename, const FileFormat _format = FileFormat::BINARY);
/// the demangled type name in a file's header ("xerus::Tensor", "xerus::TensorNetwork", "xerus::TTNetwork<false>")
std::string file_type(const std::string& _filename);
Tensor load_tensor_from_file(const std::string& _filename);
TensorNetwork load_network_from_file(const std::string& _filename);
TTTensor load_tt_from_file(const std::string& _filename);
}  // namespace misc
}  // namespace xerus
