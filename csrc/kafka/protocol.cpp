// Kafka message encoders/decoders (see protocol.h for the version table).
#include "protocol.h"

namespace gale {
namespace kafka {

const char* error_name(int code) {
  switch (code) {
    case UNKNOWN_SERVER_ERROR: return "UNKNOWN_SERVER_ERROR";
    case NONE: return "NONE";
    case OFFSET_OUT_OF_RANGE: return "OFFSET_OUT_OF_RANGE";
    case CORRUPT_MESSAGE: return "CORRUPT_MESSAGE";
    case UNKNOWN_TOPIC_OR_PARTITION: return "UNKNOWN_TOPIC_OR_PARTITION";
    case LEADER_NOT_AVAILABLE: return "LEADER_NOT_AVAILABLE";
    case NOT_LEADER_FOR_PARTITION: return "NOT_LEADER_FOR_PARTITION";
    case REQUEST_TIMED_OUT: return "REQUEST_TIMED_OUT";
    case MESSAGE_TOO_LARGE: return "MESSAGE_TOO_LARGE";
    case NETWORK_EXCEPTION: return "NETWORK_EXCEPTION";
    case NOT_ENOUGH_REPLICAS: return "NOT_ENOUGH_REPLICAS";
    case NOT_ENOUGH_REPLICAS_AFTER_APPEND: return "NOT_ENOUGH_REPLICAS_AFTER_APPEND";
    case COORDINATOR_NOT_AVAILABLE: return "COORDINATOR_NOT_AVAILABLE";
    case NOT_COORDINATOR: return "NOT_COORDINATOR";
    case INVALID_TOPIC_EXCEPTION: return "INVALID_TOPIC_EXCEPTION";
    case RECORD_LIST_TOO_LARGE: return "RECORD_LIST_TOO_LARGE";
    case INVALID_REQUIRED_ACKS: return "INVALID_REQUIRED_ACKS";
    case ILLEGAL_GENERATION: return "ILLEGAL_GENERATION";
    case INCONSISTENT_GROUP_PROTOCOL: return "INCONSISTENT_GROUP_PROTOCOL";
    case UNKNOWN_MEMBER_ID: return "UNKNOWN_MEMBER_ID";
    case INVALID_SESSION_TIMEOUT: return "INVALID_SESSION_TIMEOUT";
    case REBALANCE_IN_PROGRESS: return "REBALANCE_IN_PROGRESS";
    case UNSUPPORTED_VERSION: return "UNSUPPORTED_VERSION";
    case TOPIC_ALREADY_EXISTS: return "TOPIC_ALREADY_EXISTS";
    case INVALID_PARTITIONS: return "INVALID_PARTITIONS";
    case INVALID_REQUEST: return "INVALID_REQUEST";
    default: return "ERROR";
  }
}

bool error_retriable(int code) {
  switch (code) {
    case CORRUPT_MESSAGE:
    case UNKNOWN_TOPIC_OR_PARTITION:
    case LEADER_NOT_AVAILABLE:
    case NOT_LEADER_FOR_PARTITION:
    case REQUEST_TIMED_OUT:
    case NETWORK_EXCEPTION:
    case NOT_ENOUGH_REPLICAS:
    case NOT_ENOUGH_REPLICAS_AFTER_APPEND:
      return true;
    default:
      return false;
  }
}

namespace {
template <typename T, typename F>
void put_array(Writer& w, const std::vector<T>& v, F f) {
  w.array_len((int32_t)v.size());
  for (const T& x : v) f(x);
}
template <typename T, typename F>
std::vector<T> get_array(Reader& r, F f) {
  const int32_t n = r.array_len();
  std::vector<T> v;
  if (n <= 0) return v;
  if ((size_t)n > r.remaining()) throw ProtocolError("array length exceeds message");
  v.reserve((size_t)n);
  for (int32_t i = 0; i < n; ++i) v.push_back(f());
  return v;
}
}  // namespace

void encode_request_header(Writer& w, const RequestHeader& h) {
  w.i16(h.api_key);
  w.i16(h.api_version);
  w.i32(h.correlation_id);
  w.str(h.client_id);
}

RequestHeader decode_request_header(Reader& r) {
  RequestHeader h;
  h.api_key = r.i16();
  h.api_version = r.i16();
  h.correlation_id = r.i32();
  r.nstr(&h.client_id);
  return h;
}

// ---- ApiVersions v0 ----
void encode_api_versions_response(Writer& w, const ApiVersionsResponse& m) {
  w.i16(m.error);
  put_array(w, m.apis, [&](const ApiVersionRange& a) {
    w.i16(a.key);
    w.i16(a.min_version);
    w.i16(a.max_version);
  });
}
ApiVersionsResponse decode_api_versions_response(Reader& r) {
  ApiVersionsResponse m;
  m.error = r.i16();
  m.apis = get_array<ApiVersionRange>(r, [&] {
    ApiVersionRange a;
    a.key = r.i16();
    a.min_version = r.i16();
    a.max_version = r.i16();
    return a;
  });
  return m;
}

// ---- Metadata v4 ----
void encode_metadata_request(Writer& w, const MetadataRequest& m) {
  if (m.all_topics) {
    w.array_len(-1);
  } else {
    put_array(w, m.topics, [&](const std::string& t) { w.str(t); });
  }
  w.i8(m.allow_auto_topic_creation ? 1 : 0);
}
MetadataRequest decode_metadata_request(Reader& r) {
  MetadataRequest m;
  const int32_t n = r.array_len();
  if (n < 0) {
    m.all_topics = true;
  } else {
    for (int32_t i = 0; i < n; ++i) m.topics.push_back(r.str());
  }
  m.allow_auto_topic_creation = r.i8() != 0;
  return m;
}
void encode_metadata_response(Writer& w, const MetadataResponse& m) {
  w.i32(m.throttle_ms);
  put_array(w, m.brokers, [&](const BrokerNode& b) {
    w.i32(b.node_id);
    w.str(b.host);
    w.i32(b.port);
    w.null_str();  // rack
  });
  w.str(m.cluster_id);
  w.i32(m.controller_id);
  put_array(w, m.topics, [&](const TopicMetadata& t) {
    w.i16(t.error);
    w.str(t.name);
    w.i8(t.internal ? 1 : 0);
    put_array(w, t.partitions, [&](const PartitionMetadata& p) {
      w.i16(p.error);
      w.i32(p.index);
      w.i32(p.leader);
      put_array(w, p.replicas, [&](int32_t x) { w.i32(x); });
      put_array(w, p.isr, [&](int32_t x) { w.i32(x); });
    });
  });
}
MetadataResponse decode_metadata_response(Reader& r) {
  MetadataResponse m;
  m.throttle_ms = r.i32();
  m.brokers = get_array<BrokerNode>(r, [&] {
    BrokerNode b;
    b.node_id = r.i32();
    b.host = r.str();
    b.port = r.i32();
    std::string rack;
    r.nstr(&rack);
    return b;
  });
  r.nstr(&m.cluster_id);
  m.controller_id = r.i32();
  m.topics = get_array<TopicMetadata>(r, [&] {
    TopicMetadata t;
    t.error = r.i16();
    t.name = r.str();
    t.internal = r.i8() != 0;
    t.partitions = get_array<PartitionMetadata>(r, [&] {
      PartitionMetadata p;
      p.error = r.i16();
      p.index = r.i32();
      p.leader = r.i32();
      p.replicas = get_array<int32_t>(r, [&] { return r.i32(); });
      p.isr = get_array<int32_t>(r, [&] { return r.i32(); });
      return p;
    });
    return t;
  });
  return m;
}

// ---- Produce v3 ----
void encode_produce_request(Writer& w, const ProduceRequest& m) {
  w.null_str();  // transactional_id
  w.i16(m.acks);
  w.i32(m.timeout_ms);
  put_array(w, m.topics, [&](const ProduceTopic& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const ProducePartition& p) {
      w.i32(p.index);
      w.bytes(p.records);
    });
  });
}
ProduceRequest decode_produce_request(Reader& r) {
  ProduceRequest m;
  std::string txn;
  r.nstr(&txn);
  m.acks = r.i16();
  m.timeout_ms = r.i32();
  m.topics = get_array<ProduceTopic>(r, [&] {
    ProduceTopic t;
    t.name = r.str();
    t.partitions = get_array<ProducePartition>(r, [&] {
      ProducePartition p;
      p.index = r.i32();
      auto br = r.bytes_ref();
      p.records_off = br.first;
      p.records_len = br.second;
      return p;
    });
    return t;
  });
  return m;
}
void encode_produce_response(Writer& w, const ProduceResponse& m) {
  put_array(w, m.topics, [&](const ProduceTopicResponse& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const ProducePartitionResponse& p) {
      w.i32(p.index);
      w.i16(p.error);
      w.i64(p.base_offset);
      w.i64(p.log_append_time);
    });
  });
  w.i32(m.throttle_ms);
}
ProduceResponse decode_produce_response(Reader& r) {
  ProduceResponse m;
  m.topics = get_array<ProduceTopicResponse>(r, [&] {
    ProduceTopicResponse t;
    t.name = r.str();
    t.partitions = get_array<ProducePartitionResponse>(r, [&] {
      ProducePartitionResponse p;
      p.index = r.i32();
      p.error = r.i16();
      p.base_offset = r.i64();
      p.log_append_time = r.i64();
      return p;
    });
    return t;
  });
  m.throttle_ms = r.i32();
  return m;
}

// ---- Fetch v4 ----
void encode_fetch_request(Writer& w, const FetchRequest& m) {
  w.i32(m.replica_id);
  w.i32(m.max_wait_ms);
  w.i32(m.min_bytes);
  w.i32(m.max_bytes);
  w.i8(m.isolation_level);
  put_array(w, m.topics, [&](const FetchTopic& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const FetchPartition& p) {
      w.i32(p.index);
      w.i64(p.fetch_offset);
      w.i32(p.max_bytes);
    });
  });
}
FetchRequest decode_fetch_request(Reader& r) {
  FetchRequest m;
  m.replica_id = r.i32();
  m.max_wait_ms = r.i32();
  m.min_bytes = r.i32();
  m.max_bytes = r.i32();
  m.isolation_level = r.i8();
  m.topics = get_array<FetchTopic>(r, [&] {
    FetchTopic t;
    t.name = r.str();
    t.partitions = get_array<FetchPartition>(r, [&] {
      FetchPartition p;
      p.index = r.i32();
      p.fetch_offset = r.i64();
      p.max_bytes = r.i32();
      return p;
    });
    return t;
  });
  return m;
}
FetchResponse decode_fetch_response(Reader& r) {
  FetchResponse m;
  m.throttle_ms = r.i32();
  m.topics = get_array<FetchTopicResponse>(r, [&] {
    FetchTopicResponse t;
    t.name = r.str();
    t.partitions = get_array<FetchPartitionResponse>(r, [&] {
      FetchPartitionResponse p;
      p.index = r.i32();
      p.error = r.i16();
      p.high_watermark = r.i64();
      p.last_stable_offset = r.i64();
      const int32_t na = r.array_len();  // aborted transactions
      for (int32_t i = 0; i < na; ++i) {
        r.i64();
        r.i64();
      }
      auto br = r.bytes_ref();
      p.records_off = br.first;
      p.records_len = br.second;
      return p;
    });
    return t;
  });
  return m;
}

// ---- ListOffsets v1 ----
void encode_list_offsets_request(Writer& w, const ListOffsetsRequest& m) {
  w.i32(m.replica_id);
  put_array(w, m.topics, [&](const ListOffsetsTopic& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const ListOffsetsPartition& p) {
      w.i32(p.index);
      w.i64(p.timestamp);
    });
  });
}
ListOffsetsRequest decode_list_offsets_request(Reader& r) {
  ListOffsetsRequest m;
  m.replica_id = r.i32();
  m.topics = get_array<ListOffsetsTopic>(r, [&] {
    ListOffsetsTopic t;
    t.name = r.str();
    t.partitions = get_array<ListOffsetsPartition>(r, [&] {
      ListOffsetsPartition p;
      p.index = r.i32();
      p.timestamp = r.i64();
      return p;
    });
    return t;
  });
  return m;
}
void encode_list_offsets_response(Writer& w, const ListOffsetsResponse& m) {
  put_array(w, m.topics, [&](const ListOffsetsTopicResponse& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const ListOffsetsPartitionResponse& p) {
      w.i32(p.index);
      w.i16(p.error);
      w.i64(p.timestamp);
      w.i64(p.offset);
    });
  });
}
ListOffsetsResponse decode_list_offsets_response(Reader& r) {
  ListOffsetsResponse m;
  m.topics = get_array<ListOffsetsTopicResponse>(r, [&] {
    ListOffsetsTopicResponse t;
    t.name = r.str();
    t.partitions = get_array<ListOffsetsPartitionResponse>(r, [&] {
      ListOffsetsPartitionResponse p;
      p.index = r.i32();
      p.error = r.i16();
      p.timestamp = r.i64();
      p.offset = r.i64();
      return p;
    });
    return t;
  });
  return m;
}

// ---- FindCoordinator v1 ----
void encode_find_coordinator_request(Writer& w, const FindCoordinatorRequest& m) {
  w.str(m.key);
  w.i8(m.key_type);
}
FindCoordinatorRequest decode_find_coordinator_request(Reader& r) {
  FindCoordinatorRequest m;
  m.key = r.str();
  m.key_type = r.i8();
  return m;
}
void encode_find_coordinator_response(Writer& w, const FindCoordinatorResponse& m) {
  w.i32(m.throttle_ms);
  w.i16(m.error);
  if (m.error_message.empty()) w.null_str(); else w.str(m.error_message);
  w.i32(m.node.node_id);
  w.str(m.node.host);
  w.i32(m.node.port);
}
FindCoordinatorResponse decode_find_coordinator_response(Reader& r) {
  FindCoordinatorResponse m;
  m.throttle_ms = r.i32();
  m.error = r.i16();
  r.nstr(&m.error_message);
  m.node.node_id = r.i32();
  m.node.host = r.str();
  m.node.port = r.i32();
  return m;
}

// ---- JoinGroup v2 ----
void encode_join_group_request(Writer& w, const JoinGroupRequest& m) {
  w.str(m.group_id);
  w.i32(m.session_timeout_ms);
  w.i32(m.rebalance_timeout_ms);
  w.str(m.member_id);
  w.str(m.protocol_type);
  put_array(w, m.protocols, [&](const GroupProtocol& p) {
    w.str(p.name);
    w.bytes(p.metadata);
  });
}
JoinGroupRequest decode_join_group_request(Reader& r) {
  JoinGroupRequest m;
  m.group_id = r.str();
  m.session_timeout_ms = r.i32();
  m.rebalance_timeout_ms = r.i32();
  m.member_id = r.str();
  m.protocol_type = r.str();
  m.protocols = get_array<GroupProtocol>(r, [&] {
    GroupProtocol p;
    p.name = r.str();
    const auto b = r.bytes_ref();
    if (b.second > 0) p.metadata.assign(reinterpret_cast<const char*>(r.base() + b.first),
                                        (size_t)b.second);
    return p;
  });
  return m;
}
void encode_join_group_response(Writer& w, const JoinGroupResponse& m) {
  w.i32(m.throttle_ms);
  w.i16(m.error);
  w.i32(m.generation_id);
  w.str(m.protocol);
  w.str(m.leader_id);
  w.str(m.member_id);
  put_array(w, m.members, [&](const GroupMemberMeta& x) {
    w.str(x.member_id);
    w.bytes(x.metadata);
  });
}
namespace {
GroupMemberMeta get_member_meta(Reader& r) {
  GroupMemberMeta x;
  x.member_id = r.str();
  const auto b = r.bytes_ref();
  if (b.second > 0) x.metadata.assign(reinterpret_cast<const char*>(r.base() + b.first),
                                      (size_t)b.second);
  return x;
}
}  // namespace
JoinGroupResponse decode_join_group_response(Reader& r) {
  JoinGroupResponse m;
  m.throttle_ms = r.i32();
  m.error = r.i16();
  m.generation_id = r.i32();
  m.protocol = r.str();
  m.leader_id = r.str();
  m.member_id = r.str();
  m.members = get_array<GroupMemberMeta>(r, [&] { return get_member_meta(r); });
  return m;
}

// ---- SyncGroup v1 ----
void encode_sync_group_request(Writer& w, const SyncGroupRequest& m) {
  w.str(m.group_id);
  w.i32(m.generation_id);
  w.str(m.member_id);
  put_array(w, m.assignments, [&](const GroupMemberMeta& x) {
    w.str(x.member_id);
    w.bytes(x.metadata);
  });
}
SyncGroupRequest decode_sync_group_request(Reader& r) {
  SyncGroupRequest m;
  m.group_id = r.str();
  m.generation_id = r.i32();
  m.member_id = r.str();
  m.assignments = get_array<GroupMemberMeta>(r, [&] { return get_member_meta(r); });
  return m;
}
void encode_sync_group_response(Writer& w, const SyncGroupResponse& m) {
  w.i32(m.throttle_ms);
  w.i16(m.error);
  w.bytes(m.assignment);
}
SyncGroupResponse decode_sync_group_response(Reader& r) {
  SyncGroupResponse m;
  m.throttle_ms = r.i32();
  m.error = r.i16();
  const auto b = r.bytes_ref();
  if (b.second > 0) m.assignment.assign(reinterpret_cast<const char*>(r.base() + b.first),
                                        (size_t)b.second);
  return m;
}

// ---- Heartbeat v1 / LeaveGroup v1 ----
void encode_heartbeat_request(Writer& w, const HeartbeatRequest& m) {
  w.str(m.group_id);
  w.i32(m.generation_id);
  w.str(m.member_id);
}
HeartbeatRequest decode_heartbeat_request(Reader& r) {
  HeartbeatRequest m;
  m.group_id = r.str();
  m.generation_id = r.i32();
  m.member_id = r.str();
  return m;
}
void encode_leave_group_request(Writer& w, const LeaveGroupRequest& m) {
  w.str(m.group_id);
  w.str(m.member_id);
}
LeaveGroupRequest decode_leave_group_request(Reader& r) {
  LeaveGroupRequest m;
  m.group_id = r.str();
  m.member_id = r.str();
  return m;
}
void encode_group_error_response(Writer& w, int16_t error) {
  w.i32(0);
  w.i16(error);
}
int16_t decode_group_error_response(Reader& r) {
  r.i32();
  return r.i16();
}

// ---- ConsumerProtocol v0 (Subscription / Assignment) ----
std::string encode_subscription(const ConsumerSubscription& m) {
  Writer w;
  w.i16(0);
  put_array(w, m.topics, [&](const std::string& t) { w.str(t); });
  w.bytes(m.user_data);
  return w.buf;
}
ConsumerSubscription decode_subscription(const std::string& b) {
  Reader r(b);
  ConsumerSubscription m;
  r.i16();  // version (later versions only append fields)
  m.topics = get_array<std::string>(r, [&] { return r.str(); });
  if (r.remaining() >= 4) {
    const auto u = r.bytes_ref();
    if (u.second > 0) m.user_data = b.substr(u.first, (size_t)u.second);
  }
  return m;
}
std::string encode_assignment(const ConsumerAssignment& m) {
  Writer w;
  w.i16(0);
  put_array(w, m.partitions, [&](const std::pair<std::string, std::vector<int32_t>>& tp) {
    w.str(tp.first);
    put_array(w, tp.second, [&](int32_t p) { w.i32(p); });
  });
  w.bytes(m.user_data);
  return w.buf;
}
ConsumerAssignment decode_assignment(const std::string& b) {
  ConsumerAssignment m;
  if (b.empty()) return m;  // no partitions for this member
  Reader r(b);
  r.i16();
  m.partitions = get_array<std::pair<std::string, std::vector<int32_t>>>(r, [&] {
    std::pair<std::string, std::vector<int32_t>> tp;
    tp.first = r.str();
    tp.second = get_array<int32_t>(r, [&] { return r.i32(); });
    return tp;
  });
  if (r.remaining() >= 4) {
    const auto u = r.bytes_ref();
    if (u.second > 0) m.user_data = b.substr(u.first, (size_t)u.second);
  }
  return m;
}

// ---- OffsetCommit v2 ----
void encode_offset_commit_request(Writer& w, const OffsetCommitRequest& m) {
  w.str(m.group_id);
  w.i32(m.generation_id);
  w.str(m.member_id);
  w.i64(m.retention_ms);
  put_array(w, m.topics, [&](const CommitTopic& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const CommitPartition& p) {
      w.i32(p.index);
      w.i64(p.offset);
      w.str(p.metadata);
    });
  });
}
OffsetCommitRequest decode_offset_commit_request(Reader& r) {
  OffsetCommitRequest m;
  m.group_id = r.str();
  m.generation_id = r.i32();
  m.member_id = r.str();
  m.retention_ms = r.i64();
  m.topics = get_array<CommitTopic>(r, [&] {
    CommitTopic t;
    t.name = r.str();
    t.partitions = get_array<CommitPartition>(r, [&] {
      CommitPartition p;
      p.index = r.i32();
      p.offset = r.i64();
      r.nstr(&p.metadata);
      return p;
    });
    return t;
  });
  return m;
}
void encode_offset_commit_response(Writer& w, const std::vector<CommitTopic>& topics) {
  put_array(w, topics, [&](const CommitTopic& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const CommitPartition& p) {
      w.i32(p.index);
      w.i16(p.error);
    });
  });
}
std::vector<CommitTopic> decode_offset_commit_response(Reader& r) {
  return get_array<CommitTopic>(r, [&] {
    CommitTopic t;
    t.name = r.str();
    t.partitions = get_array<CommitPartition>(r, [&] {
      CommitPartition p;
      p.index = r.i32();
      p.error = r.i16();
      return p;
    });
    return t;
  });
}

// ---- OffsetFetch v1 ----
void encode_offset_fetch_request(Writer& w, const OffsetFetchRequest& m) {
  w.str(m.group_id);
  put_array(w, m.topics, [&](const CommitTopic& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const CommitPartition& p) { w.i32(p.index); });
  });
}
OffsetFetchRequest decode_offset_fetch_request(Reader& r) {
  OffsetFetchRequest m;
  m.group_id = r.str();
  m.topics = get_array<CommitTopic>(r, [&] {
    CommitTopic t;
    t.name = r.str();
    t.partitions = get_array<CommitPartition>(r, [&] {
      CommitPartition p;
      p.index = r.i32();
      return p;
    });
    return t;
  });
  return m;
}
void encode_offset_fetch_response(Writer& w, const std::vector<CommitTopic>& topics) {
  put_array(w, topics, [&](const CommitTopic& t) {
    w.str(t.name);
    put_array(w, t.partitions, [&](const CommitPartition& p) {
      w.i32(p.index);
      w.i64(p.offset);
      w.str(p.metadata);
      w.i16(p.error);
    });
  });
}
std::vector<CommitTopic> decode_offset_fetch_response(Reader& r) {
  return get_array<CommitTopic>(r, [&] {
    CommitTopic t;
    t.name = r.str();
    t.partitions = get_array<CommitPartition>(r, [&] {
      CommitPartition p;
      p.index = r.i32();
      p.offset = r.i64();
      r.nstr(&p.metadata);
      p.error = r.i16();
      return p;
    });
    return t;
  });
}

// ---- CreateTopics v2 ----
void encode_create_topics_request(Writer& w, const CreateTopicsRequest& m) {
  put_array(w, m.topics, [&](const CreateTopic& t) {
    w.str(t.name);
    w.i32(t.partitions);
    w.i16(t.replication_factor);
    w.array_len(0);  // manual assignments
    w.array_len(0);  // configs
  });
  w.i32(m.timeout_ms);
  w.i8(m.validate_only ? 1 : 0);
}
CreateTopicsRequest decode_create_topics_request(Reader& r) {
  CreateTopicsRequest m;
  m.topics = get_array<CreateTopic>(r, [&] {
    CreateTopic t;
    t.name = r.str();
    t.partitions = r.i32();
    t.replication_factor = r.i16();
    const int32_t na = r.array_len();
    for (int32_t i = 0; i < na; ++i) {
      r.i32();
      const int32_t nb = r.array_len();
      for (int32_t j = 0; j < nb; ++j) r.i32();
    }
    const int32_t nc = r.array_len();
    for (int32_t i = 0; i < nc; ++i) {
      r.str();
      std::string v;
      r.nstr(&v);
    }
    return t;
  });
  m.timeout_ms = r.i32();
  m.validate_only = r.i8() != 0;
  return m;
}
void encode_create_topics_response(Writer& w, const std::vector<CreateTopic>& topics) {
  w.i32(0);  // throttle
  put_array(w, topics, [&](const CreateTopic& t) {
    w.str(t.name);
    w.i16(t.error);
    if (t.error_message.empty()) w.null_str(); else w.str(t.error_message);
  });
}
std::vector<CreateTopic> decode_create_topics_response(Reader& r) {
  r.i32();
  return get_array<CreateTopic>(r, [&] {
    CreateTopic t;
    t.name = r.str();
    t.error = r.i16();
    r.nstr(&t.error_message);
    return t;
  });
}

}  // namespace kafka
}  // namespace gale
