// Consumer-group coordinator of the embedded broker: JoinGroup / SyncGroup / Heartbeat /
// LeaveGroup with Kafka's eager rebalance protocol, plus generation fencing of OffsetCommit.
//
// The reference scales and heals through Storm: the spout tasks split the partitions (E1) and
// supervisors restart dead workers (E4). gale's elastic equivalent is Kafka's own
// group membership: every serving process joins one group; when a member joins, leaves or stops
// heartbeating for session_timeout_ms, the coordinator moves the group to PreparingRebalance,
// the surviving members rejoin, the leader (a client) computes the new partition assignment and
// distributes it through SyncGroup, and each member resumes its new partitions from the
// committed offsets. Like Kafka's GroupCoordinator:
//   Empty -> PreparingRebalance -> CompletingRebalance -> Stable (-> PreparingRebalance ...)
// Requests block their connection thread (the broker serves one thread per connection): a
// JoinGroup returns once every known member has rejoined or the rebalance timeout expired, a
// SyncGroup once the leader delivered the assignment.
#pragma once
#include <stdint.h>

#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "protocol.h"

namespace gale {
namespace kafka {

struct GroupInfo {
  std::string state;
  int32_t generation = 0;
  std::string leader, protocol;
  std::vector<std::string> members;
};

class GroupCoordinator {
 public:
  JoinGroupResponse join(const JoinGroupRequest& req, const std::string& client_id);
  SyncGroupResponse sync(const SyncGroupRequest& req);
  int16_t heartbeat(const HeartbeatRequest& req);
  int16_t leave(const LeaveGroupRequest& req);
  // OffsetCommit fencing: generation < 0 (a simple, group-less commit) always passes
  int16_t check_commit(const std::string& group, int32_t generation, const std::string& member);
  GroupInfo describe(const std::string& group);
  void shutdown();  // wake every blocked request (broker stop)

 private:
  struct Member {
    std::string id, client_id;
    std::vector<GroupProtocol> protocols;
    int32_t session_ms = 10000, rebalance_ms = 30000;
    int64_t last_seen = 0;
    int64_t order = 0;    // join order (the leader is the longest-standing member)
    bool joined = false;  // has (re)joined the rebalance in progress
    int waiting = 0;      // requests of this member blocked in JoinGroup / SyncGroup right now
    std::string assignment;
  };
  struct Group {
    std::string state = "Empty";
    int32_t generation = 0;
    std::string protocol, leader;
    std::map<std::string, Member> members;
    int64_t deadline = 0;  // PreparingRebalance: rebalance timeout
    bool synced = false;   // CompletingRebalance: the leader's assignment arrived
    std::condition_variable cv;
  };
  Group& group(const std::string& id);
  void expire(Group& g, int64_t now);
  void prepare(Group& g, int64_t now);
  bool complete_join(Group& g);  // false: no member left
  std::mutex mu_;
  std::map<std::string, std::unique_ptr<Group>> groups_;
  int64_t next_id_ = 0;
  bool closed_ = false;
};

}  // namespace kafka
}  // namespace gale
