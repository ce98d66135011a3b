%% psim_strategy_harness -- the in-BEAM parity harness for the pluggable
%% manager's membership strategies (SURVEY.md App. C, 8(f3); VERDICT r2
%% item 4): the reference's own strategy modules
%%   partisan_full_membership_strategy      (full:42-144)
%%   partisan_scamp_v1_membership_strategy  (scamp_v1:45-279)
%%   partisan_scamp_v2_membership_strategy  (scamp_v2:57-360)
%% run unmodified for N simulated nodes inside ONE BEAM process, called
%% exactly where partisan_pluggable_peer_service_manager calls them
%% (pl = src/partisan_pluggable_peer_service_manager.erl):
%%   Strategy:init/1           init/1 (pl:384)
%%   Strategy:join/3           handle_info({connected, Node, _, RemoteState}) (pl:986-1044)
%%   Strategy:periodic/1       handle_info(periodic) (pl:881-903)
%%   Strategy:handle_message/2 handle_message({membership_strategy, M}) (pl:1153-1195)
%%   Strategy:leave/2          internal_leave/2 (pl:1390-1420)
%% under the simulator's round model R0-P (DESIGN.md section 2b).  The
%% manager's glue around those calls is restated here, as the oracle
%% restates it (oracle/psim_oracle.c pl_process_node): the hello / state
%% handshake of internal_join/3 (pl:1423-1458, peer_service_server:125-148),
%% establish_connections/3 (pl:1096-1108: a send succeeds iff the peer is a
%% member or the pending contact, runs, and no partition separates them), the
%% dispatch draw of a successful send (util:190-195), the stop when a
%% handle_message result leaves the node out of its own membership
%% (pl:1182-1188), with that round's sends undone (they were casts to
%% itself, pl:1585-1609).  Every emitted message is written as a record line
%% in the engine's encoding (the oracle's pl_emit), so compare_trace.py can
%% diff the stream against the CPU oracle -- and through it the GPU engine.
%%
%% Scope: the reference semantics only -- fanout 0 (the full strategy
%% gossips to every member; config B's fanout > 0 is the simulator's
%% extension of a key no strategy reads, App. A Q10), no omission faults.
%% SCAMP's isolation test reads erlang:timestamp(); the harness sets
%% last_message_time before periodic/1 so that it reads "isolated" exactly
%% when the oracle's round model does (a ping was ever received, none this
%% round; App. A Q12): 1 s ago, now, or undefined.
%%
%% NOT RUN HERE: this image has no Erlang VM (SURVEY 8(c)).  Run recipe:
%% erlang/harness/README.md (scenario names ending in _pl).
-module(psim_strategy_harness).
-export([main/1, run/2]).

-define(NONE, 16#FFFFFFFF).
%% message types of a PLUGGABLE handle (include/partisan_gpu_sim.h psim_pl_msg_type)
-define(HELLO, 0).
-define(STATE, 1).
-define(GOSSIP, 2).
-define(FWD_SUB, 3).
-define(PING, 4).
-define(KEEP_SUB, 5).
-define(REMOVE_SUB, 6).
-define(BOOT_REMOVE, 7).
%% position of last_message_time in the SCAMP records (scamp_v1:36, scamp_v2:44-47)
-define(V1_LAST, 4).
-define(V2_LAST, 5).

%% erl -noshell -pa shims -pa <partisan ebin> -pa . -s psim_strategy_harness main Scenario Out
main([Scenario, Out]) ->
    {ok, Events} = file:consult(atom_to_list(Scenario)),
    ok = run(Events, atom_to_list(Out)),
    halt(0).

%% Events (file:consult terms): as psim_harness, with
%%   {config, #{n_nodes, seed, rounds, strategy := full | scamp_v1 | scamp_v2,
%%              periodic_interval => 10, scamp_c => 5}}
%%   {leave, Round, [{Actor, Target}]}       leave/1 at Actor (pl:502-515)
run(Events, OutFile) ->
    [Cfg] = [C || {config, C} <- Events],
    #{n_nodes := N, seed := Seed, rounds := Rounds, strategy := Strategy} = Cfg,
    put(psim_h_n, N),
    put(psim_h_seed, Seed),
    put(psim_h_part, maps:new()),
    put(psim_s_mod, module(Strategy)),
    put(psim_s_kind, Strategy),
    put(psim_s_period, maps:get(periodic_interval, Cfg, 10)),
    [put({psim_h_cfg, K}, V) || {K, V} <- maps:to_list(maps:without([n_nodes, seed, rounds, strategy], Cfg))],
    put({psim_h_cfg, random_seed_int}, Seed),
    {ok, F} = file:open(OutFile, [write]),
    Nodes = lists:foldl(fun(R, Acc) -> round(R, Events, Acc, F) end, #{}, lists:seq(0, Rounds - 1)),
    %% the sets v1 buckets SCAMP v1's membership set is ordered by (App. A Q1)
    ok = psim_harness:write_buckets(F, N),
    [io:format(F, "V ~b ~s~n", [Id, string:join([integer_to_list(psim_harness:id_of(P)) || P <- M], " ")])
     || {Id, #{up := true, members := M}} <- lists:sort(maps:to_list(Nodes))],
    file:close(F).

module(full) -> partisan_full_membership_strategy;
module(scamp_v1) -> partisan_scamp_v1_membership_strategy;
module(scamp_v2) -> partisan_scamp_v2_membership_strategy.

%% ----------------------------------------------------------- one round
round(R, Events, Nodes0, F) ->
    put(psim_h_round, R),
    put(psim_h_out, []),
    put(psim_h_seq, #{}),
    Crashed = lists:append([Ids || {crash, RR, Ids} <- Events, RR =:= R]),
    Nodes1 = lists:foldl(fun(Id, Acc) -> set_up(Id, false, Acc) end, Nodes0, Crashed),
    [put(psim_h_part, maps:from_list(lists:zip(lists:seq(0, get(psim_h_n) - 1), G)))
     || {partition, RR, G} <- Events, RR =:= R],
    [put(psim_h_part, maps:new()) || {clear_partition, RR} <- Events, RR =:= R],
    Starts = lists:append([J || {join, RR, J} <- Events, RR =:= R]),
    Nodes2 = lists:foldl(fun({Id, C}, Acc) -> start(Id, C, R, Acc) end, Nodes1, Starts),
    Leaves = maps:from_list(lists:append([L || {leave, RR, L} <- Events, RR =:= R])),
    Inbox = get(psim_s_inbox_next, #{}),
    put(psim_h_nodes, Nodes2),
    {Nodes3, Stopped} =
        lists:foldl(fun(Id, {Acc, St}) ->
                            case maps:get(Id, Acc) of
                                #{up := true} = Node ->
                                    put(psim_h_nodes, Acc),
                                    case node_round(Id, Node, R, maps:get(Id, Inbox, []), maps:get(Id, Leaves, none), Acc) of
                                        {ok, Node1} -> {Acc#{Id => Node1}, St};
                                        stop -> {Acc, [Id | St]}
                                    end;
                                _ -> {Acc, St}
                            end
                    end, {Nodes2, []}, lists:sort(maps:keys(Nodes2))),
    %% managers that stopped are down from the next round (psim_leave_node)
    Nodes4 = lists:foldl(fun(Id, Acc) -> set_up(Id, false, Acc) end, Nodes3, Stopped),
    Out = lists:reverse(get(psim_h_out)),
    [io:format(F, "R ~b ~b ~b ~b ~b 0 ~b 0 0 0~n", [R, S, Q, D, T, A0])
     || {S, Q, D, {T, A0}, _Msg} <- Out],
    put(psim_s_inbox_next,
        lists:foldl(fun({_S, _Q, D, _Rec, Msg}, Acc) ->
                            maps:update_with(D, fun(L) -> L ++ [Msg] end, [Msg], Acc)
                    end, #{}, Out)),
    Nodes4.

node_round(Id, Node0, R, Msgs0, Leave, Nodes) ->
    #{st := S0, ctr := Ctr0, start := Start} = Node0,
    Mod = get(psim_s_mod),
    put(psim_h_node, Id),
    psim_philox:install(get(psim_h_seed), Id, Ctr0),
    Msgs = case Start =:= R of true -> []; false -> Msgs0 end,   % a fresh incarnation drops its inbox
    Out0 = get(psim_h_out),
    Seq0 = get(psim_h_seq),
    N1 = case Leave of                                 % leave/1, before the hello and the inbox
             none -> Node0;
             T -> {ok, M, Outgoing, S1} = Mod:leave(S0, psim_harness:spec(T)),
                  send_all(Id, Outgoing, Node0#{st := S1, members := M})
         end,
    N2 = case maps:get(pending, N1) of                 % internal_join/3: connect, hello
             none -> N1;
             C -> case maps:get(hello_sent, N1) of
                      true -> N1;
                      false -> case psim_harness:reachable(Id, C) of
                                   true -> record(Id, C, {?HELLO, 0}, {hello, Id}), N1#{hello_sent := true};
                                   false -> N1
                               end
                  end
         end,
    case inbox(Id, Msgs, N2, R, Nodes) of
        stop ->
            put(psim_h_out, Out0),                     % its sends were casts to itself
            put(psim_h_seq, Seq0),
            stop;
        N3 ->
            N4 = case due(get(psim_s_period), R, Start) of
                     true -> {ok, M2, Outgoing2, S2} = Mod:periodic(isolation(N3, R)),
                             send_all(Id, Outgoing2, N3#{st := S2, members := M2});
                     false -> N3
                 end,
            {_, _, Ctr} = psim_philox:state(),
            {ok, N4#{ctr := Ctr}}
    end.

inbox(_Id, [], N, _R, _Nodes) -> N;
inbox(Id, [{hello, From} | Rest], N, R, Nodes) ->
    %% the contact's server answers with get_local_state/0 (server:125-148)
    case psim_harness:reachable(Id, From) of
        true -> record(Id, From, {?STATE, state_count(maps:get(st, N))}, {state, Id, maps:get(st, N)});
        false -> ok
    end,
    inbox(Id, Rest, N, R, Nodes);
inbox(Id, [{state, From, Remote} | Rest], N, R, Nodes) ->
    case maps:get(pending, N) of
        From ->
            {ok, M, Outgoing, S1} = (get(psim_s_mod)):join(maps:get(st, N), psim_harness:spec(From), Remote),
            inbox(Id, Rest, send_all(Id, Outgoing, N#{st := S1, members := M, pending := none}), R, Nodes);
        _ -> inbox(Id, Rest, N, R, Nodes)
    end;
inbox(Id, [{membership_strategy, Msg} | Rest], N, R, Nodes) ->
    N1 = case Msg of {ping, _} -> N#{pinged := R}; _ -> N end,
    %% a strategy that raises crashes its manager (scamp_v1:197's swapped
    %% sets:del_element/2 arguments, scamp_v2:213's lists:nth(0, ..), App. A
    %% Q12): a stop, as the oracle's
    try (get(psim_s_mod)):handle_message(maps:get(st, N1), Msg) of
        {ok, M, Outgoing, S1} ->
            case lists:member(psim_harness:spec(Id), M) of
                false -> stop;                         % pl:1182-1188
                true -> inbox(Id, Rest, send_all(Id, Outgoing, N1#{st := S1, members := M}), R, Nodes)
            end
    catch
        _:_ -> stop
    end.

%% the outgoing list, in order (pl: schedule_self_message_delivery, then
%% do_send_message/7 :1309-1363)
send_all(Id, Outgoing, N) ->
    lists:foreach(fun({Peer, Msg}) -> send(Id, psim_harness:id_of(Peer), Msg, N) end, Outgoing),
    N.

send(Id, Dst, Msg, N) ->
    Member = lists:any(fun(P) -> psim_harness:id_of(P) =:= Dst end, maps:get(members, N)),
    Full = get(psim_s_kind) =:= full,
    case psim_harness:reachable(Id, Dst) andalso (Full orelse Member orelse maps:get(pending, N) =:= Dst) of
        true ->
            _ = rand:uniform(1),                       % dispatch_pid/3 (util:190-195)
            record(Id, Dst, enc(Msg), Msg);
        false -> ok
    end.

record(Src, Dst, Rec, Msg) ->
    Seqs = get(psim_h_seq),
    Q = maps:get(Src, Seqs, 0),
    put(psim_h_seq, Seqs#{Src => Q + 1}),
    put(psim_h_out, [{Src, Q, Dst, Rec, Msg} | get(psim_h_out)]).

%% the oracle's record fields {Type, A0} (psim_oracle.c pl_emit call sites)
enc({membership_strategy, {forward_subscription, Node}}) -> {?FWD_SUB, psim_harness:id_of(Node)};
enc({membership_strategy, {ping, Node}}) -> {?PING, psim_harness:id_of(Node)};
enc({membership_strategy, {keep_subscription, Node}}) -> {?KEEP_SUB, psim_harness:id_of(Node)};
enc({membership_strategy, {remove_subscription, Node}}) -> {?REMOVE_SUB, psim_harness:id_of(Node)};
enc({membership_strategy, {bootstrap_remove_subscription, Node}}) -> {?BOOT_REMOVE, psim_harness:id_of(Node)};
enc({membership_strategy, {#{name := _}, State}}) -> {?GOSSIP, state_count(State)}.

%% the member count a full-strategy state carries (0 for SCAMP)
state_count(State) when element(1, State) =:= full_v1 ->
    length(sets:to_list(state_orset:query(element(3, State))));
state_count(_) -> 0.

%% SCAMP's isolation window read from erlang:timestamp() (App. A Q12): the
%% oracle's "a ping was ever received, none this round"
isolation(N, R) ->
    S = maps:get(st, N),
    Pos = case element(1, S) of scamp_v1 -> ?V1_LAST; scamp_v2 -> ?V2_LAST; _ -> none end,
    case {Pos, maps:get(pinged, N)} of
        {none, _} -> S;
        {_, never} -> setelement(Pos, S, undefined);
        {_, R} -> setelement(Pos, S, erlang:timestamp());
        {_, _} -> {M, Sec, U} = erlang:timestamp(), setelement(Pos, S, {M, Sec - 1, U})
    end.

due(Period, R, Start) -> R > Start andalso (R - Start) rem Period =:= 0.

start(Id, Contact, R, Nodes) ->
    put(psim_h_node, Id),
    Mod = get(psim_s_mod),
    psim_philox:install(get(psim_h_seed), Id, 0),
    {ok, M, S} = Mod:init(psim_harness:name(Id)),   % (the manager's gen_actor/0 stand-in)
    {_, _, Ctr} = psim_philox:state(),
    C = case Contact of none -> none; ?NONE -> none; _ -> Contact end,
    Nodes#{Id => #{st => S, members => M, ctr => Ctr, start => R, pending => C, hello_sent => false,
                   up => true, pinged => never}}.

set_up(Id, Up, Nodes) ->
    case maps:get(Id, Nodes, undefined) of
        undefined -> Nodes;
        N -> Nodes#{Id := N#{up := Up}}
    end.
