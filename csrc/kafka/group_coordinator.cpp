// Consumer-group coordinator (see group_coordinator.h).
#include "group_coordinator.h"

#include <algorithm>
#include <chrono>

namespace gale {
namespace kafka {

namespace {
int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
std::chrono::steady_clock::time_point at_ms(int64_t ms) {
  return std::chrono::steady_clock::time_point(std::chrono::milliseconds(ms));
}
}  // namespace

GroupCoordinator::Group& GroupCoordinator::group(const std::string& id) {
  auto& g = groups_[id];
  if (!g) g = std::make_unique<Group>();
  return *g;
}

// Members whose session lapsed leave the group; a stable group then rebalances. As in Kafka, a
// member blocked in JoinGroup / SyncGroup (or already rejoined while the group prepares a
// rebalance) is not expired: it is waiting on the coordinator, not silent. Members that never
// rejoin are dropped by complete_join at the rebalance deadline instead.
void GroupCoordinator::expire(Group& g, int64_t now) {
  bool gone = false;
  for (auto it = g.members.begin(); it != g.members.end();) {
    const Member& m = it->second;
    const bool exempt = m.waiting > 0 || (g.state == "PreparingRebalance" && m.joined);
    if (!exempt && now - m.last_seen > m.session_ms) {
      if (g.leader == it->first) g.leader.clear();
      it = g.members.erase(it);
      gone = true;
    } else {
      ++it;
    }
  }
  if (!gone) return;
  if (g.members.empty()) {
    g.state = "Empty";
  } else if (g.state != "PreparingRebalance") {
    prepare(g, now);
  }
  g.cv.notify_all();
}

void GroupCoordinator::prepare(Group& g, int64_t now) {
  g.state = "PreparingRebalance";
  int32_t rb = 0;
  for (auto& kv : g.members) {
    kv.second.joined = false;
    rb = std::max(rb, kv.second.rebalance_ms);
  }
  g.deadline = now + rb;
  g.synced = false;
}

bool GroupCoordinator::complete_join(Group& g) {
  for (auto it = g.members.begin(); it != g.members.end();)
    it = it->second.joined ? std::next(it) : g.members.erase(it);  // missed the rebalance
  if (g.members.empty()) {
    g.state = "Empty";
    g.leader.clear();
    return false;
  }
  // the protocol every member supports, in the leader's order of preference
  if (g.leader.empty() || !g.members.count(g.leader)) {
    const Member* first = nullptr;
    for (auto& kv : g.members)
      if (!first || kv.second.order < first->order) first = &kv.second;
    g.leader = first->id;
  }
  g.protocol.clear();
  for (const GroupProtocol& p : g.members[g.leader].protocols) {
    bool all = true;
    for (auto& kv : g.members) {
      bool has = false;
      for (const GroupProtocol& q : kv.second.protocols) has |= q.name == p.name;
      all &= has;
    }
    if (all) {
      g.protocol = p.name;
      break;
    }
  }
  ++g.generation;
  g.state = "CompletingRebalance";
  g.synced = false;
  // every survivor's session restarts now (its JoinGroup answer is on its way; a member whose
  // thread has not woken yet must not be expired by another request in the meantime)
  const int64_t now = now_ms();
  for (auto& kv : g.members) {
    kv.second.assignment.clear();
    kv.second.last_seen = now;
  }
  g.cv.notify_all();
  return true;
}

JoinGroupResponse GroupCoordinator::join(const JoinGroupRequest& req, const std::string& client_id) {
  JoinGroupResponse resp;
  std::unique_lock<std::mutex> lk(mu_);
  if (closed_) {
    resp.error = COORDINATOR_NOT_AVAILABLE;
    return resp;
  }
  if (req.session_timeout_ms < 1 || req.session_timeout_ms > 1800000 || req.protocols.empty()) {
    resp.error = req.protocols.empty() ? INCONSISTENT_GROUP_PROTOCOL : INVALID_SESSION_TIMEOUT;
    return resp;
  }
  Group& g = group(req.group_id);
  int64_t now = now_ms();
  expire(g, now);
  std::string id = req.member_id;
  if (id.empty()) {
    id = (client_id.empty() ? std::string("member") : client_id) + "-" + std::to_string(++next_id_);
  } else if (!g.members.count(id)) {
    resp.error = UNKNOWN_MEMBER_ID;  // fenced (its session expired): rejoin as a new member
    return resp;
  }
  const bool fresh = !g.members.count(id);
  Member& m = g.members[id];
  if (fresh) m.order = ++next_id_;
  m.id = id;
  m.client_id = client_id;
  m.protocols = req.protocols;
  m.session_ms = req.session_timeout_ms;
  m.rebalance_ms = std::max(req.rebalance_timeout_ms, 1);
  m.last_seen = now;
  if (g.state != "PreparingRebalance") prepare(g, now);
  g.deadline = std::max(g.deadline, now + m.rebalance_ms);
  m.joined = true;
  g.cv.notify_all();
  const int32_t gen0 = g.generation;
  ++m.waiting;
  while (g.generation == gen0 && !closed_) {
    bool all = true;
    for (auto& kv : g.members) all &= kv.second.joined;
    now = now_ms();
    if (all || now >= g.deadline) {
      complete_join(g);
      break;
    }
    g.cv.wait_until(lk, at_ms(std::min(g.deadline, now + 100)));
  }
  auto it = g.members.find(id);
  if (it != g.members.end()) --it->second.waiting;
  if (closed_ || it == g.members.end() || g.generation == gen0) {
    resp.error = closed_ ? COORDINATOR_NOT_AVAILABLE : UNKNOWN_MEMBER_ID;
    return resp;
  }
  it->second.last_seen = now_ms();
  if (g.protocol.empty()) {
    resp.error = INCONSISTENT_GROUP_PROTOCOL;
    return resp;
  }
  resp.generation_id = g.generation;
  resp.protocol = g.protocol;
  resp.leader_id = g.leader;
  resp.member_id = id;
  if (id == g.leader) {
    for (auto& kv : g.members) {
      GroupMemberMeta mm;
      mm.member_id = kv.first;
      for (const GroupProtocol& p : kv.second.protocols)
        if (p.name == g.protocol) mm.metadata = p.metadata;
      resp.members.push_back(std::move(mm));
    }
  }
  return resp;
}

SyncGroupResponse GroupCoordinator::sync(const SyncGroupRequest& req) {
  SyncGroupResponse resp;
  std::unique_lock<std::mutex> lk(mu_);
  Group& g = group(req.group_id);
  expire(g, now_ms());
  auto it = g.members.find(req.member_id);
  if (it == g.members.end()) {
    resp.error = UNKNOWN_MEMBER_ID;
    return resp;
  }
  if (g.state == "PreparingRebalance") {
    resp.error = REBALANCE_IN_PROGRESS;
    return resp;
  }
  if (req.generation_id != g.generation) {
    resp.error = ILLEGAL_GENERATION;
    return resp;
  }
  it->second.last_seen = now_ms();
  if (req.member_id == g.leader && g.state == "CompletingRebalance") {
    const int64_t now = now_ms();
    for (auto& kv : g.members) kv.second.last_seen = now;  // (sessions restart with the answer)
    for (const GroupMemberMeta& a : req.assignments) {
      auto m = g.members.find(a.member_id);
      if (m != g.members.end()) m->second.assignment = a.metadata;
    }
    g.synced = true;
    g.state = "Stable";
    g.cv.notify_all();
  }
  const int32_t gen = g.generation;
  const int64_t deadline = now_ms() + it->second.rebalance_ms;
  ++it->second.waiting;
  while (!closed_ && g.generation == gen && !g.synced && g.state == "CompletingRebalance" &&
         now_ms() < deadline)
    g.cv.wait_until(lk, at_ms(std::min(deadline, now_ms() + 100)));
  it = g.members.find(req.member_id);
  if (it != g.members.end()) --it->second.waiting;
  if (closed_ || it == g.members.end()) {
    resp.error = closed_ ? COORDINATOR_NOT_AVAILABLE : UNKNOWN_MEMBER_ID;
  } else if (g.generation != gen || !g.synced) {
    resp.error = REBALANCE_IN_PROGRESS;
  } else {
    it->second.last_seen = now_ms();
    resp.assignment = it->second.assignment;
  }
  return resp;
}

int16_t GroupCoordinator::heartbeat(const HeartbeatRequest& req) {
  std::lock_guard<std::mutex> lk(mu_);
  Group& g = group(req.group_id);
  const int64_t now = now_ms();
  auto it = g.members.find(req.member_id);
  if (it != g.members.end()) it->second.last_seen = now;  // (before expiring the others)
  expire(g, now);
  if (closed_) return COORDINATOR_NOT_AVAILABLE;
  if (!g.members.count(req.member_id)) return UNKNOWN_MEMBER_ID;
  if (g.state == "PreparingRebalance") return REBALANCE_IN_PROGRESS;
  if (req.generation_id != g.generation) return ILLEGAL_GENERATION;
  return NONE;
}

int16_t GroupCoordinator::leave(const LeaveGroupRequest& req) {
  std::lock_guard<std::mutex> lk(mu_);
  Group& g = group(req.group_id);
  if (!g.members.erase(req.member_id)) return UNKNOWN_MEMBER_ID;
  if (g.leader == req.member_id) g.leader.clear();
  if (g.members.empty()) g.state = "Empty";
  else if (g.state != "PreparingRebalance") prepare(g, now_ms());
  g.cv.notify_all();
  return NONE;
}

int16_t GroupCoordinator::check_commit(const std::string& group_id, int32_t generation,
                                       const std::string& member) {
  if (generation < 0) return NONE;
  std::lock_guard<std::mutex> lk(mu_);
  auto git = groups_.find(group_id);
  if (git == groups_.end()) return ILLEGAL_GENERATION;
  Group& g = *git->second;
  auto it = g.members.find(member);
  if (it == g.members.end()) return UNKNOWN_MEMBER_ID;
  if (generation != g.generation) return ILLEGAL_GENERATION;
  it->second.last_seen = now_ms();
  return NONE;
}

GroupInfo GroupCoordinator::describe(const std::string& group_id) {
  std::lock_guard<std::mutex> lk(mu_);
  GroupInfo gi;
  auto git = groups_.find(group_id);
  if (git == groups_.end()) {
    gi.state = "Dead";
    return gi;
  }
  Group& g = *git->second;
  expire(g, now_ms());
  gi.state = g.state;
  gi.generation = g.generation;
  gi.leader = g.leader;
  gi.protocol = g.protocol;
  for (auto& kv : g.members) gi.members.push_back(kv.first);
  return gi;
}

void GroupCoordinator::shutdown() {
  std::lock_guard<std::mutex> lk(mu_);
  closed_ = true;
  for (auto& kv : groups_) kv.second->cv.notify_all();
}

}  // namespace kafka
}  // namespace gale
