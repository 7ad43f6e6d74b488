// Kafka request/response messages spoken by gale's client and embedded broker.
//
// One (non-flexible) version per API, chosen to be accepted by Kafka 2.x through 4.x brokers
// (KIP-896 removed only older versions):
//   ApiVersions v0, Metadata v4, Produce v3, Fetch v4, ListOffsets v1, FindCoordinator v1,
//   OffsetCommit v2, OffsetFetch v1, CreateTopics v2, and the consumer-group membership APIs
//   JoinGroup v2, SyncGroup v1, Heartbeat v1, LeaveGroup v1 (with the "consumer" embedded
//   protocol's Subscription / Assignment v0 encodings).
// The client checks them against the broker's ApiVersions answer before use.
//
// Reference mapping: Metadata/Fetch/ListOffsets = KafkaSpout partition
// discovery and reads (E1, MainTopology.java:95-106); OffsetCommit/OffsetFetch = the spout's ZK
// offset commits (X3); Produce = KafkaProducer.send (E7, KafkaBolt.java:144). The group APIs
// replace Storm's supervisor/rebalance machinery for consumers (E4): members of
// one group share the input partitions and a dead member's partitions move to the survivors.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "wire.h"

namespace gale {
namespace kafka {

enum ApiKey : int16_t {
  PRODUCE = 0,
  FETCH = 1,
  LIST_OFFSETS = 2,
  METADATA = 3,
  OFFSET_COMMIT = 8,
  OFFSET_FETCH = 9,
  FIND_COORDINATOR = 10,
  JOIN_GROUP = 11,
  HEARTBEAT = 12,
  LEAVE_GROUP = 13,
  SYNC_GROUP = 14,
  API_VERSIONS = 18,
  CREATE_TOPICS = 19,
};

constexpr int16_t kVersion(ApiKey k) {
  return k == PRODUCE ? 3 : k == FETCH ? 4 : k == LIST_OFFSETS ? 1 : k == METADATA ? 4
       : k == OFFSET_COMMIT ? 2 : k == OFFSET_FETCH ? 1 : k == FIND_COORDINATOR ? 1
       : k == API_VERSIONS ? 0 : k == CREATE_TOPICS ? 2 : k == JOIN_GROUP ? 2
       : k == HEARTBEAT ? 1 : k == LEAVE_GROUP ? 1 : k == SYNC_GROUP ? 1 : -1;
}

enum ErrorCode : int16_t {
  UNKNOWN_SERVER_ERROR = -1,
  NONE = 0,
  OFFSET_OUT_OF_RANGE = 1,
  CORRUPT_MESSAGE = 2,
  UNKNOWN_TOPIC_OR_PARTITION = 3,
  LEADER_NOT_AVAILABLE = 5,
  NOT_LEADER_FOR_PARTITION = 6,
  REQUEST_TIMED_OUT = 7,
  MESSAGE_TOO_LARGE = 10,
  NETWORK_EXCEPTION = 13,
  COORDINATOR_NOT_AVAILABLE = 15,
  NOT_COORDINATOR = 16,
  INVALID_TOPIC_EXCEPTION = 17,
  RECORD_LIST_TOO_LARGE = 18,
  NOT_ENOUGH_REPLICAS = 19,
  NOT_ENOUGH_REPLICAS_AFTER_APPEND = 20,
  INVALID_REQUIRED_ACKS = 21,
  ILLEGAL_GENERATION = 22,
  INCONSISTENT_GROUP_PROTOCOL = 23,
  UNKNOWN_MEMBER_ID = 25,
  INVALID_SESSION_TIMEOUT = 26,
  REBALANCE_IN_PROGRESS = 27,
  UNSUPPORTED_VERSION = 35,
  TOPIC_ALREADY_EXISTS = 36,
  INVALID_PARTITIONS = 37,
  INVALID_REQUEST = 42,
};

const char* error_name(int code);
// Kafka's RetriableException family (kafka-clients Errors): a produce that failed with one of
// these may succeed when sent again (leader moved, broker busy, connection lost)
bool error_retriable(int code);

// ListOffsets special timestamps
constexpr int64_t kLatest = -1;
constexpr int64_t kEarliest = -2;

struct RequestHeader {
  int16_t api_key = 0;
  int16_t api_version = 0;
  int32_t correlation_id = 0;
  std::string client_id;
};

void encode_request_header(Writer& w, const RequestHeader& h);
RequestHeader decode_request_header(Reader& r);

// ---- ApiVersions ----
struct ApiVersionRange {
  int16_t key, min_version, max_version;
};
struct ApiVersionsResponse {
  int16_t error = 0;
  std::vector<ApiVersionRange> apis;
};
void encode_api_versions_response(Writer& w, const ApiVersionsResponse& m);
ApiVersionsResponse decode_api_versions_response(Reader& r);

// ---- Metadata v4 ----
struct MetadataRequest {
  bool all_topics = false;
  std::vector<std::string> topics;
  bool allow_auto_topic_creation = true;
};
struct BrokerNode {
  int32_t node_id = 0;
  std::string host;
  int32_t port = 0;
};
struct PartitionMetadata {
  int16_t error = 0;
  int32_t index = 0;
  int32_t leader = -1;
  std::vector<int32_t> replicas, isr;
};
struct TopicMetadata {
  int16_t error = 0;
  std::string name;
  bool internal = false;
  std::vector<PartitionMetadata> partitions;
};
struct MetadataResponse {
  int32_t throttle_ms = 0;
  std::vector<BrokerNode> brokers;
  std::string cluster_id;
  int32_t controller_id = -1;
  std::vector<TopicMetadata> topics;
};
void encode_metadata_request(Writer& w, const MetadataRequest& m);
MetadataRequest decode_metadata_request(Reader& r);
void encode_metadata_response(Writer& w, const MetadataResponse& m);
MetadataResponse decode_metadata_response(Reader& r);

// ---- Produce v3 ----
struct ProducePartition {
  int32_t index = 0;
  std::string records;            // encoded RecordBatch(es) (client side)
  size_t records_off = 0;         // decoded (broker side): offset into the request buffer
  int32_t records_len = -1;
};
struct ProduceTopic {
  std::string name;
  std::vector<ProducePartition> partitions;
};
struct ProduceRequest {
  int16_t acks = 1;
  int32_t timeout_ms = 30000;
  std::vector<ProduceTopic> topics;
};
struct ProducePartitionResponse {
  int32_t index = 0;
  int16_t error = 0;
  int64_t base_offset = -1;
  int64_t log_append_time = -1;
};
struct ProduceTopicResponse {
  std::string name;
  std::vector<ProducePartitionResponse> partitions;
};
struct ProduceResponse {
  std::vector<ProduceTopicResponse> topics;
  int32_t throttle_ms = 0;
};
void encode_produce_request(Writer& w, const ProduceRequest& m);
ProduceRequest decode_produce_request(Reader& r);  // records referenced, not copied
void encode_produce_response(Writer& w, const ProduceResponse& m);
ProduceResponse decode_produce_response(Reader& r);

// ---- Fetch v4 ----
struct FetchPartition {
  int32_t index = 0;
  int64_t fetch_offset = 0;
  int32_t max_bytes = 1 << 20;
};
struct FetchTopic {
  std::string name;
  std::vector<FetchPartition> partitions;
};
struct FetchRequest {
  int32_t replica_id = -1;
  int32_t max_wait_ms = 500;
  int32_t min_bytes = 1;
  int32_t max_bytes = 50 << 20;
  int8_t isolation_level = 0;
  std::vector<FetchTopic> topics;
};
struct FetchPartitionResponse {
  int32_t index = 0;
  int16_t error = 0;
  int64_t high_watermark = -1;
  int64_t last_stable_offset = -1;
  size_t records_off = 0;  // into the response buffer
  int32_t records_len = -1;
};
struct FetchTopicResponse {
  std::string name;
  std::vector<FetchPartitionResponse> partitions;
};
struct FetchResponse {
  int32_t throttle_ms = 0;
  std::vector<FetchTopicResponse> topics;
};
void encode_fetch_request(Writer& w, const FetchRequest& m);
FetchRequest decode_fetch_request(Reader& r);
FetchResponse decode_fetch_response(Reader& r);  // (the broker encodes it zero-copy itself)

// ---- ListOffsets v1 ----
struct ListOffsetsPartition {
  int32_t index = 0;
  int64_t timestamp = kLatest;
};
struct ListOffsetsTopic {
  std::string name;
  std::vector<ListOffsetsPartition> partitions;
};
struct ListOffsetsRequest {
  int32_t replica_id = -1;
  std::vector<ListOffsetsTopic> topics;
};
struct ListOffsetsPartitionResponse {
  int32_t index = 0;
  int16_t error = 0;
  int64_t timestamp = -1;
  int64_t offset = -1;
};
struct ListOffsetsTopicResponse {
  std::string name;
  std::vector<ListOffsetsPartitionResponse> partitions;
};
struct ListOffsetsResponse {
  std::vector<ListOffsetsTopicResponse> topics;
};
void encode_list_offsets_request(Writer& w, const ListOffsetsRequest& m);
ListOffsetsRequest decode_list_offsets_request(Reader& r);
void encode_list_offsets_response(Writer& w, const ListOffsetsResponse& m);
ListOffsetsResponse decode_list_offsets_response(Reader& r);

// ---- FindCoordinator v1 ----
struct FindCoordinatorRequest {
  std::string key;
  int8_t key_type = 0;  // 0 = group
};
struct FindCoordinatorResponse {
  int32_t throttle_ms = 0;
  int16_t error = 0;
  std::string error_message;
  BrokerNode node;
};
void encode_find_coordinator_request(Writer& w, const FindCoordinatorRequest& m);
FindCoordinatorRequest decode_find_coordinator_request(Reader& r);
void encode_find_coordinator_response(Writer& w, const FindCoordinatorResponse& m);
FindCoordinatorResponse decode_find_coordinator_response(Reader& r);

// ---- OffsetCommit v2 / OffsetFetch v1 ----
struct CommitPartition {
  int32_t index = 0;
  int64_t offset = -1;
  std::string metadata;
  int16_t error = 0;
};
struct CommitTopic {
  std::string name;
  std::vector<CommitPartition> partitions;
};
struct OffsetCommitRequest {
  std::string group_id;
  int32_t generation_id = -1;
  std::string member_id;
  int64_t retention_ms = -1;
  std::vector<CommitTopic> topics;
};
void encode_offset_commit_request(Writer& w, const OffsetCommitRequest& m);
OffsetCommitRequest decode_offset_commit_request(Reader& r);
void encode_offset_commit_response(Writer& w, const std::vector<CommitTopic>& topics);
std::vector<CommitTopic> decode_offset_commit_response(Reader& r);

struct OffsetFetchRequest {
  std::string group_id;
  std::vector<CommitTopic> topics;  // partition indexes only
};
void encode_offset_fetch_request(Writer& w, const OffsetFetchRequest& m);
OffsetFetchRequest decode_offset_fetch_request(Reader& r);
void encode_offset_fetch_response(Writer& w, const std::vector<CommitTopic>& topics);
std::vector<CommitTopic> decode_offset_fetch_response(Reader& r);

// ---- group membership: JoinGroup v2 / SyncGroup v1 / Heartbeat v1 / LeaveGroup v1 ----
struct GroupProtocol {
  std::string name;      // assignor ("range", "roundrobin")
  std::string metadata;  // consumer Subscription
};
struct JoinGroupRequest {
  std::string group_id;
  int32_t session_timeout_ms = 10000;
  int32_t rebalance_timeout_ms = 30000;
  std::string member_id;  // empty on the first join
  std::string protocol_type = "consumer";
  std::vector<GroupProtocol> protocols;
};
struct GroupMemberMeta {
  std::string member_id;
  std::string metadata;
};
struct JoinGroupResponse {
  int32_t throttle_ms = 0;
  int16_t error = 0;
  int32_t generation_id = -1;
  std::string protocol;  // the chosen assignor
  std::string leader_id;
  std::string member_id;
  std::vector<GroupMemberMeta> members;  // leader only
};
void encode_join_group_request(Writer& w, const JoinGroupRequest& m);
JoinGroupRequest decode_join_group_request(Reader& r);
void encode_join_group_response(Writer& w, const JoinGroupResponse& m);
JoinGroupResponse decode_join_group_response(Reader& r);

struct SyncGroupRequest {
  std::string group_id;
  int32_t generation_id = -1;
  std::string member_id;
  std::vector<GroupMemberMeta> assignments;  // leader only: member -> Assignment bytes
};
struct SyncGroupResponse {
  int32_t throttle_ms = 0;
  int16_t error = 0;
  std::string assignment;
};
void encode_sync_group_request(Writer& w, const SyncGroupRequest& m);
SyncGroupRequest decode_sync_group_request(Reader& r);
void encode_sync_group_response(Writer& w, const SyncGroupResponse& m);
SyncGroupResponse decode_sync_group_response(Reader& r);

struct HeartbeatRequest {
  std::string group_id;
  int32_t generation_id = -1;
  std::string member_id;
};
void encode_heartbeat_request(Writer& w, const HeartbeatRequest& m);
HeartbeatRequest decode_heartbeat_request(Reader& r);
struct LeaveGroupRequest {
  std::string group_id;
  std::string member_id;
};
void encode_leave_group_request(Writer& w, const LeaveGroupRequest& m);
LeaveGroupRequest decode_leave_group_request(Reader& r);
// Heartbeat v1 / LeaveGroup v1 responses: throttle_time_ms, error_code
void encode_group_error_response(Writer& w, int16_t error);
int16_t decode_group_error_response(Reader& r);

// "consumer" embedded protocol (Kafka's ConsumerProtocol v0)
struct ConsumerSubscription {
  std::vector<std::string> topics;
  std::string user_data;
};
struct ConsumerAssignment {
  std::vector<std::pair<std::string, std::vector<int32_t>>> partitions;
  std::string user_data;
};
std::string encode_subscription(const ConsumerSubscription& m);
ConsumerSubscription decode_subscription(const std::string& b);
std::string encode_assignment(const ConsumerAssignment& m);
ConsumerAssignment decode_assignment(const std::string& b);

// ---- CreateTopics v2 ----
struct CreateTopic {
  std::string name;
  int32_t partitions = 1;
  int16_t replication_factor = 1;
  int16_t error = 0;
  std::string error_message;
};
struct CreateTopicsRequest {
  std::vector<CreateTopic> topics;
  int32_t timeout_ms = 30000;
  bool validate_only = false;
};
void encode_create_topics_request(Writer& w, const CreateTopicsRequest& m);
CreateTopicsRequest decode_create_topics_request(Reader& r);
void encode_create_topics_response(Writer& w, const std::vector<CreateTopic>& topics);
std::vector<CreateTopic> decode_create_topics_response(Reader& r);

}  // namespace kafka
}  // namespace gale
